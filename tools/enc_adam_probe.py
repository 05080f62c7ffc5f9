"""Timing probe (results INVALID): bench.py with the encoder half of Adam moved to the side stream after the decoder
half, unordered with the next step's G1 (engine.ENC_ADAM_SIDE_PROBE) -- the upper bound of what overlapping the
encoder-half Adam with G1 could save (profiles/r05_enc_adam_overlap_bound.txt).  The switch lived in engine.py only
for the measurement: run this in a tree of commit c23c73f (tools/snapshot_head.sh c23c73f).
Usage: python tools/enc_adam_probe.py [bench.py args]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import crosscoder_amd.engine as engine  # noqa: E402

if not hasattr(engine, "ENC_ADAM_SIDE_PROBE"):
    sys.exit("tools/enc_adam_probe.py: this engine has no ENC_ADAM_SIDE_PROBE switch; use a tree of commit c23c73f")
engine.ENC_ADAM_SIDE_PROBE = True
import bench  # noqa: E402

sys.argv = ["bench.py"] + sys.argv[1:]
sys.exit(bench.main())
