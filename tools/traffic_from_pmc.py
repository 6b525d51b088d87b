"""Turn two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of one bench run into
profiles/<round>/<config>_traffic.json (HBM bytes per replay launch).

usage: python tools/traffic_from_pmc.py FETCH_CSV WRITE_CSV OUT_JSON CONFIG DOCS MSGS [KERNEL[+KERNEL...]]
traffic = 2*FETCH_SIZE + WRITE_SIZE: the gfx950 one-half FETCH_SIZE correction of
/opt/skills/guides/MI355X_MICROARCH.md (HBM section); counters are taken at the
L2 memory side, so Infinity-Cache hits are included.
"""
import csv
import json
import re
import sys


def bare(name):
    """'void mt_replay_blk_kernel<false>(MtState, ...)' -> 'mt_replay_blk_kernel'."""
    return re.split(r"[<(]", re.sub(r"^void ", "", name.strip()))[0]


def per_launch(path, counter, kernel="mt_replay_kernel"):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if bare(r["Kernel_Name"]) == kernel and r["Counter_Name"] == counter]
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} in {path}")
    return sum(vals) / len(vals) * 1024.0  # rocprofv3 reports kB


def main():
    fcsv, wcsv, out, cfg, docs, msgs = sys.argv[1:7]
    kernel = sys.argv[7] if len(sys.argv) > 7 else "mt_replay_blk_kernel"
    # KERNEL may name several kernels joined by "+" (one replay launch made of several, e.g.
    # config 5's partitioned size classes): their per-launch bytes are summed
    ks = kernel.split("+")
    fetch = sum(per_launch(fcsv, "FETCH_SIZE", k) for k in ks)
    write = sum(per_launch(wcsv, "WRITE_SIZE", k) for k in ks)
    rec = {"kernel": kernel, "workload": cfg, "docs": int(docs), "msgs_per_doc": int(msgs),
           "fetch_bytes_raw": fetch, "write_bytes": write, "traffic_bytes": 2 * fetch + write,
           "note": "per launch; rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of "
                   "`bench.py --steps 1 --warmup 0 --no-cpu-baseline`; traffic = 2*FETCH_SIZE + WRITE_SIZE"}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
