#!/usr/bin/env python3
"""Hello-world Actor (reference ``examples/aloha_honua/aloha_honua_0.py``).

    python -m aiko_services_amd.tools.mqtt broker &          # in-repo MQTT broker
    python -m aiko_services_amd.tools.registrar &
    python -m aiko_services_amd.examples.aloha_honua.aloha_honua_0 &
    python -m aiko_services_amd.tools.mqtt pub <topic printed above> "(aloha Pele)"
"""
import aiko_services_amd as aiko


class AlohaHonua(aiko.Actor):
    def __init__(self, context):
        context.get_implementation("Actor").__init__(self, context)
        self.greetings = 0
        print(f"MQTT topic: {self.topic_in}", flush=True)

    def aloha(self, name):
        self.greetings += 1
        self.share["greetings"] = self.greetings
        self.logger.info(f"Aloha {name} !")


def main():
    aiko.compose_instance(AlohaHonua, aiko.actor_args("aloha_honua"))
    aiko.process.run()


if __name__ == "__main__":
    main()
