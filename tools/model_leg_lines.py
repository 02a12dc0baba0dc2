"""CPU model (MEASUREMENTS.md, round 5): how many distinct 16-lane state lines a
64-source block's derived-row legs touch on C3, with root lanes numbered in slot
order (the library's) or by first reference from the legs.  Uses the derivation
rule and slot order restated in tools/model_share_closure.py.

    python tools/model_leg_lines.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from model_share_closure import model  # noqa: E402


def main(n: int = 50000):
    order, derived, legs = model(n)
    roots = [int(v) for v in order if not derived[v]]
    lane_slot = {v: i for i, v in enumerate(roots)}
    lane_ref = {}
    for v in order:
        v = int(v)
        for r in ([v] if not derived[v] else sorted(legs[v])):
            lane_ref.setdefault(r, len(lane_ref))

    def stats(lane):
        lines, refs = [], 0
        for b in range(0, n, 64):
            rr = []
            for v in (int(x) for x in order[b:b + 64]):
                rr += [v] if not derived[v] else list(legs[v])
            refs += len(rr)
            lines.append(len({lane[r] // 16 for r in rr}))
        return float(np.mean(lines)), refs / (n / 64)

    for name, lane in (("slot order", lane_slot), ("first reference", lane_ref)):
        ln, rf = stats(lane)
        print(f"lanes by {name}: {ln:.1f} distinct lines per block for {rf:.1f} leg references")


if __name__ == "__main__":
    main()
