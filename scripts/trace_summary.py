"""Steady-state kernel summary from a rocprofv3 kernel trace.

``python scripts/trace_summary.py <kernel_trace.csv> [--steps K] [--top N]``: keeps the
kernels launched after the LAST marker kernel (bench.py launches ``torch.cuda._sleep``
right before its timed region when ``GARFIELD_TRACE_MARK=1``), so MIOpen's find/tuning
kernels of the warm-up steps do not pollute the table, and prints per-kernel totals per
step plus the busy/idle split of the timed window."""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--marker", default="spin")
    ap.add_argument("--json", default="", help="also write {kernel: {ms_per_step, calls_per_step}} here")
    ap.add_argument("--sequence", default="", help="also write the last step's dispatches (start offset, "
                    "duration, kernel) to this file")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    cut = 0
    for i, (_, _, name) in enumerate(rows):
        if a.marker in name.lower():
            cut = i + 1
    rows = rows[cut:]
    if not rows:
        raise SystemExit("no kernels after the marker")
    agg = defaultdict(lambda: [0, 0])
    busy = 0
    last_end = rows[0][0]
    for s, e, name in rows:
        short = name.replace("(anonymous namespace)::", "").split("(")[0][:110]
        agg[short][0] += 1
        agg[short][1] += e - s
        busy += max(0, e - max(s, last_end))
        last_end = max(last_end, e)
    window = rows[-1][1] - rows[0][0]
    total = sum(v[1] for v in agg.values())
    k = max(a.steps, 1)
    print(f"kernels after marker: {len(rows)} ({len(rows) / k:.0f}/step); window {window / 1e6 / k:.3f} ms/step; "
          f"GPU busy {busy / 1e6 / k:.3f} ms/step ({100 * busy / max(window, 1):.1f}%)")
    print(f"{'ms/step':>9} {'%':>6} {'calls/step':>10}  kernel")
    for name, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[: a.top]:
        print(f"{t / 1e6 / k:9.3f} {100 * t / total:6.2f} {c / k:10.1f}  {name}")
    if a.json:
        import json
        with open(a.json, "w") as fh:
            json.dump({n: {"ms_per_step": t / 1e6 / k, "calls_per_step": c / k} for n, (c, t) in agg.items()}
                      | {"__window__": {"ms_per_step": window / 1e6 / k, "busy_ms_per_step": busy / 1e6 / k}},
                      fh, indent=1)
    if a.sequence:
        last = rows[-(len(rows) // k):]
        t0 = last[0][0]
        with open(a.sequence, "w") as fh:
            fh.write(f"{'start_us':>9} {'dur_us':>8}  kernel\n")
            for s, e, name in last:
                short = name.replace("(anonymous namespace)::", "").split("(")[0][:90]
                fh.write(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {short}\n")


if __name__ == "__main__":
    main()
