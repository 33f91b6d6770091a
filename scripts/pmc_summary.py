"""Steady-state per-kernel counter totals from a rocprofv3 ``--pmc`` run.

``python scripts/pmc_summary.py <counter_collection.csv> --steps K [--json out.json]``
keeps the dispatches after the LAST marker kernel (bench.py launches ``torch.cuda._sleep``
right before its timed region when ``GARFIELD_TRACE_MARK=1``), sums every counter per
kernel name and divides by the step count.  The JSON it writes is what
``scripts/roofline.py`` joins with the kernel-time summary."""
import argparse
import csv
import json
from collections import defaultdict


def short_name(name: str) -> str:
    return name.replace("(anonymous namespace)::", "").split("(")[0][:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--marker", default="spin")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as fh:
        for r in csv.DictReader(fh):
            did = int(r.get("Dispatch_Id") or r.get("Correlation_Id") or 0)
            rows.append((did, r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"])))
    rows.sort(key=lambda t: t[0])
    cut = -1
    for did, name, _, _ in rows:
        if a.marker in name.lower():
            cut = did
    rows = [t for t in rows if t[0] > cut]
    if not rows:
        raise SystemExit("no dispatches after the marker")
    k = max(a.steps, 1)
    agg = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for did, name, cname, val in rows:
        s = short_name(name)
        agg[s][cname] += val / k
        disp[s].add(did)
    out = {s: dict(v, dispatches_per_step=len(disp[s]) / k) for s, v in agg.items()}
    counters = sorted({c for v in agg.values() for c in v})
    print(f"{len(out)} kernels after marker; counters: {', '.join(counters)}")
    for s, v in sorted(out.items(), key=lambda kv: -sum(x for c, x in kv[1].items() if c != "dispatches_per_step"))[:40]:
        vals = " ".join(f"{c}={v.get(c, 0):.4g}" for c in counters)
        print(f"{vals}  {s}")
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
