"""Models built only from aiko_services_amd HIP ops (random-init weights)."""
