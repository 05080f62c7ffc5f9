"""Fixture loading helpers (fixtures are data written by tools/gen_golden.py)."""
import glob
import json
import os

import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def step_fixtures():
    return sorted(os.path.basename(p)[:-3] for p in glob.glob(os.path.join(GOLDEN, "*.pt"))
                  if not os.path.basename(p).startswith("buffer"))


def load(name):
    rec = torch.load(os.path.join(GOLDEN, name + ".pt"), weights_only=True)
    rec["cfg"] = json.loads(rec["cfg"])
    return rec
