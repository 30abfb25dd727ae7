"""Multi-process load-test elements."""
