"""Reduce one rocprofv3 SQ PMC pass of a bench run to the replay kernel's wave-cycle split and
instruction mix (per launch).

usage: python tools/sq_mix.py SQ_CSV [KERNEL]
SQ_WAVE_CYCLES / SQ_WAIT_ANY (parked on s_waitcnt or a barrier) / SQ_WAIT_INST_ANY (issue stall)
/ SQ_ACTIVE_INST_ANY (issuing) count quad-cycles summed over waves (MI355X_MICROARCH.md, PMC
section: the last three are disjoint and add up to about the first); SQ_INSTS_* count wave
instructions.
"""
import csv
import sys
from collections import defaultdict

from traffic_from_pmc import bare


def main():
    path = sys.argv[1]
    kernel = sys.argv[2] if len(sys.argv) > 2 else "mt_replay_blk_kernel"
    tot, launches = defaultdict(float), defaultdict(set)
    for r in csv.DictReader(open(path)):
        if bare(r["Kernel_Name"]) == kernel:
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            launches[r["Counter_Name"]].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
    if not tot:
        raise SystemExit(f"no rows for {kernel} in {path}")
    n = max(len(v) for v in launches.values()) or 1
    wc = tot.get("SQ_WAVE_CYCLES", 0.0)
    print(f"{kernel}: {n} launch(es); per launch:")
    for k in sorted(tot):
        v = tot[k] / n
        share = f"  ({100.0 * tot[k] / wc:5.1f} % of wave cycles)" if k.startswith(("SQ_WAIT", "SQ_ACTIVE")) and wc else ""
        print(f"  {k:22s} {v:16.0f}{share}")
    insts = sum(tot[k] for k in tot if k.startswith("SQ_INSTS_")) / n
    if insts and wc:
        print(f"  wave quad-cycles per counted instruction: {wc / n / insts:.2f}")


if __name__ == "__main__":
    main()
