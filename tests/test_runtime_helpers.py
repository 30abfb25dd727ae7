"""Helper implementations loaded by dotted path from tests (Interface.default targets)."""


class GreeterImpl:
    def greet(self, name):
        return f"default {name}"

