"""L7 element library: media I/O (host) and GPU elements (device-resident)."""
