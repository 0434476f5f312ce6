"""Writes tests/golden/testdukeconfig_schema.json: the pipelines of the reference's own
config file (/root/reference/src/main/resources/testdukeconfig.xml) as parsed by
dukehip.config.parse_microservice_config (ConfigLoader semantics, App.java:264-281,
291-293, 407-411, 613-647).  The fixture is the parsed schema data (properties,
comparators, low/high, thresholds, data-source columns), not the XML text, so the GPU box
(which has no /root/reference) can run the reference's schema.

    python tests/gen_reference_schema.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sesam-duke-microservice_amd"))
REF_XML = "/root/reference/src/main/resources/testdukeconfig.xml"
OUT = os.path.join(ROOT, "tests", "golden", "testdukeconfig_schema.json")


def parsed(path=REF_XML):
    from dukehip.config import parse_microservice_config
    with open(path) as f:
        cfgs = parse_microservice_config(f.read())
    return {f"{kind}/{name}": c.to_dict() for (kind, name), c in sorted(cfgs.items())}


if __name__ == "__main__":
    with open(OUT, "w") as f:
        json.dump({"source": "src/main/resources/testdukeconfig.xml", "pipelines": parsed()}, f,
                  indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", OUT)
