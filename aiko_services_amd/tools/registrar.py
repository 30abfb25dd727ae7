"""``aiko_registrar`` console entry: run a Registrar service (see control/registrar.py)."""
from aiko_services_amd.control.registrar import main

if __name__ == "__main__":
    main()
