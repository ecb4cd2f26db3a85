#!/usr/bin/env python3
"""Cross-XCD hand-off probe numbers (mp4x.ops.coherence.xcd_probe, csrc/runtime/xcd_probe.hip):
for each fence mask, how many 16-byte vectors a consumer workgroup read stale after a producer on
another XCD overwrote them.  One JSON line per mask.

    python bench/coherence_probe.py [--rounds 200] [--region-vecs 256]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=200)
    ap.add_argument("--region-vecs", type=int, default=256)
    a = ap.parse_args()
    import torch
    from mp4x.ops.coherence import NO_ACQUIRE, NO_RELEASE, xcd_probe
    torch.cuda.set_device(0)
    names = {0: "fenced", NO_RELEASE: "no_release", NO_ACQUIRE: "no_acquire", NO_RELEASE | NO_ACQUIRE: "no_fences"}
    for mask, name in names.items():
        r = xcd_probe(rounds=a.rounds, mask=mask, region_vecs=a.region_vecs)
        r["name"] = name
        r["stale_fraction"] = round(r["stale"] / (a.rounds * r["vectors_per_round"]), 4)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
