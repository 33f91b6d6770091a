"""Overlap evidence from a rocprofv3 kernel trace of ``bench.py --shard-gar`` with
GARFIELD_LOOPBACK_EXCHANGE=1: for the last timed step, the side-stream bucket copies
(the emulated all-to-all) versus the grouped backward's kernels. A copy that starts
before the backward's last kernel ends ran UNDER the backward (overlap)."""
import csv
import sys


def main():
    rows = []
    with open(sys.argv[1]) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Stream_Id", "")))
    rows.sort()
    cut = max((i for i, r in enumerate(rows) if "spin" in r[2].lower()), default=-1) + 1
    rows = rows[cut:]
    # step boundaries: the cross-entropy forward kernel starts each grouped step's loss
    xent = [i for i, r in enumerate(rows) if "xent" in r[2].lower() and "bwd" not in r[2].lower()]
    first = xent[-1] if xent else 0
    step = rows[first:]
    copies = [r for r in step if "copy" in r[2].lower() or "elementwise_kernel" in r[2].lower()]
    gemm = [r for r in step if any(k in r[2].lower() for k in ("iconv", "iwgrad", "gemm", "col2im", "bn_"))]
    if not gemm:
        print("no backward kernels found")
        return
    bwd_end = max(r[1] for r in gemm)
    t0 = step[0][0]
    print(f"step window: {(step[-1][1] - t0) / 1e3:.1f} us, last backward-class kernel ends at {(bwd_end - t0) / 1e3:.1f} us")
    under = 0
    for s, e, name, sid in copies:
        ov = s < bwd_end
        under += ov
        print(f"  {'OVERLAP' if ov else 'after  '} copy start {(s - t0) / 1e3:9.1f} us dur {(e - s) / 1e3:7.1f} us "
              f"stream {sid} {name.split('(')[0][:70]}")
    print(f"copies under the backward: {under} of {len(copies)}")


if __name__ == "__main__":
    main()
