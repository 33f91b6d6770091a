"""Per-kernel stall / occupancy table of the bench step from one SQ counter pass.

``python scripts/stall_table.py times.json stalls.json [--md out.md] [--top 12]``

times.json: ``trace_summary.py --json`` (steady-state ms and launches per step); stalls.json:
``pmc_summary.py --json`` of a pass with SQ_WAVES, SQ_WAVE_CYCLES, SQ_WAIT_ANY, SQ_WAIT_INST_ANY,
SQ_ACTIVE_INST_ANY, SQ_LDS_BANK_CONFLICT, SQ_LDS_IDX_ACTIVE and SQ_BUSY_CYCLES. Per kernel:

* wave-cycle split (MI355X_MICROARCH.md "rocprofv3 PMC slots": the three are disjoint and sum
  to about SQ_WAVE_CYCLES): parked on a wait (s_waitcnt / barrier), issue-stalled (MFMA / pipe
  dependency), issuing;
* resident waves per SIMD, estimated as 4 x SQ_WAVE_CYCLES (quad-cycles) / (kernel time x
  2.1 GHz x 1024 SIMDs) (the clock varies under load: MI355X_MICROARCH.md "DVFS give-back");
* LDS bank-conflict cycles as a share of all LDS-array cycles."""
import argparse
import json

CLOCK = 2.1e9
SIMDS = 256 * 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("times")
    ap.add_argument("stalls")
    ap.add_argument("--md", default="")
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    times = json.load(open(a.times))
    times.pop("__window__", None)
    cnt = json.load(open(a.stalls))
    out = ["| kernel | ms/step | launches | waves/launch | waves/SIMD (est.) | % waiting | % issue-stalled | "
           "% issuing | LDS conflict % |", "|---|---|---|---|---|---|---|---|---|"]
    for name, t in sorted(times.items(), key=lambda kv: -kv[1]["ms_per_step"])[: a.top]:
        c = cnt.get(name)
        if not c:
            continue
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        calls = t["calls_per_step"]

        def pct(k):
            return f"{100.0 * c.get(k, 0.0) / wc:.0f}" if wc > 0 else "-"

        occ = 4.0 * wc / (t["ms_per_step"] * 1e-3 * CLOCK * SIMDS) if t["ms_per_step"] > 0 else 0.0
        lds = c.get("SQ_LDS_IDX_ACTIVE", 0.0)
        ldsc = f"{100.0 * c.get('SQ_LDS_BANK_CONFLICT', 0.0) / lds:.1f}" if lds > 0 else "-"
        out.append(f"| {name[:78]} | {t['ms_per_step']:.3f} | {calls:.0f} | "
                   f"{c.get('SQ_WAVES', 0.0) / max(calls, 1e-9):.0f} | {occ:.2f} | {pct('SQ_WAIT_ANY')} | "
                   f"{pct('SQ_WAIT_INST_ANY')} | {pct('SQ_ACTIVE_INST_ANY')} | {ldsc} |")
    text = "\n".join(out)
    print(text)
    if a.md:
        with open(a.md, "w") as fh:
            fh.write(text + "\n")


if __name__ == "__main__":
    main()
