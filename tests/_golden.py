"""Load the committed golden fixtures (tests/golden/*.json.gz)."""
import gzip
import importlib
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN_DIR = os.path.join(HERE, "golden")
mapgen = importlib.import_module("network-distributed-q-learning_amd.mapgen")


def cases():
    return sorted(f[:-8] for f in os.listdir(GOLDEN_DIR) if f.endswith(".json.gz"))


def load(name):
    with gzip.open(os.path.join(GOLDEN_DIR, name + ".json.gz"), "rt") as f:
        d = json.load(f)
    d["scenario_obj"] = mapgen.Scenario.from_json(json.dumps(d["scenario"]))
    return d
