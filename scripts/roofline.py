"""Per-kernel-class roofline table of the bench step.

Joins the steady-state kernel times (``trace_summary.py --json``) with the per-kernel
counters of the ``--pmc`` passes (``pmc_summary.py --json``):

* bytes read  = 2 x FETCH_SIZE x 1 KiB (gfx950 tallies a 128-B fabric read as 64 B:
  MI355X_MICROARCH.md "HBM"), bytes written = WRITE_SIZE x 1 KiB.  Both count traffic
  past the XCD's L2 (Infinity-Cache hits included), i.e. what the kernel really moved;
* MFMA FLOPs  = 512 x SQ_INSTS_VALU_MFMA_MOPS_{BF16,F16,F32} (units of 512 FLOP).

``python scripts/roofline.py times.json pmc1.json [pmc2.json ...] [--md out.md]``
prints (and writes as Markdown) one row per kernel class and the top kernels, with
achieved TB/s and TFLOP/s and the fraction of the MI355X peaks they represent
(8 TB/s HBM spec, ~6.3 TB/s achievable; 2.5 PFLOP/s dense bf16 MFMA)."""
import argparse
import json
import re
from collections import defaultdict

HBM_PEAK = 8.0e12
HBM_ACHIEVABLE = 6.3e12
MFMA_PEAK = 2.5e15

CLASSES = [
    ("BatchNorm (partial / finalize / apply / small)", r"k_partial|k_fwd_apply|k_bwd_apply|k_bn_|finalize|bn_running"),
    ("hipBLASLt GEMM (1x1 conv, stem, layer4, classifier)", r"^Cijk_"),
    ("hand-written 1x1 / im2col GEMMs (gemm_nt.hip)", r"k_gemm_nt|k_gemm_ws"),
    ("halo-staged 3x3 conv / weight gradient (conv3x3_nhwc.hip)", r"k_conv3x3|k_wgrad3x3"),
    ("stem 7x7 (stem_nhwc.hip)", r"k_stem"),
    ("fp32 split-bf16 convolutions / weight gradients (conv_f32.hip)", r"k_cf32|k_wsplit|k_f32_"),
    ("implicit-GEMM conv fwd/dgrad (k_iconv_lds)", r"k_iconv"),
    ("implicit weight gradients (k_iwgrad)", r"k_iwgrad"),
    ("im2col / col2im", r"im2col|col2im"),
    ("max-pool", r"maxpool"),
    ("GAR (Gram / selection / coordinate rules / combine+SGD)", r"k_gram|k_select|k_combine|k_coord|k_krum|k_bulyan|"
                                                               r"k_median|k_tail|k_brute|k_aksel|k_sqdist|k_large|"
                                                               r"k_window|k_mean"),
    ("cross-entropy", r"k_xent"),
    ("fresh-batch gather / augmentation", r"k_augment"),
    ("flatten / cast / split-K sums into the exchange rows", r"flatten|cast|split_reduce"),
    ("ATen reductions / elementwise", r"at::native"),
]


def klass(name: str) -> str:
    for label, pat in CLASSES:
        if re.search(pat, name):
            return label
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("times")
    ap.add_argument("pmc", nargs="+")
    ap.add_argument("--md", default="")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    times = json.load(open(a.times))
    window = times.pop("__window__", {})
    cnt = defaultdict(dict)
    for p in a.pmc:
        for k, v in json.load(open(p)).items():
            cnt[k].update(v)
    rows = []
    for k, t in times.items():
        c = cnt.get(k, {})
        rd = 2.0 * 1024.0 * c["FETCH_SIZE"] if "FETCH_SIZE" in c else None
        wr = 1024.0 * c["WRITE_SIZE"] if "WRITE_SIZE" in c else None
        mops = [c[x] for x in ("SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_INSTS_VALU_MFMA_MOPS_F16",
                               "SQ_INSTS_VALU_MFMA_MOPS_F32") if x in c]
        fl = 512.0 * sum(mops) if mops else None
        rows.append(dict(name=k, cls=klass(k), ms=t["ms_per_step"], calls=t["calls_per_step"], rd=rd, wr=wr, fl=fl))

    def fmt_rate(b, ms):
        return f"{b / (ms * 1e-3) / 1e12:.2f}" if (b is not None and ms > 0) else "-"

    def line(label, ms, calls, rd, wr, fl):
        by = (rd or 0) + (wr or 0) if (rd is not None or wr is not None) else None
        tbs = by / (ms * 1e-3) if by is not None and ms > 0 else None
        tfs = fl / (ms * 1e-3) if fl is not None and ms > 0 else None
        return (f"| {label} | {ms:.3f} | {calls:.0f} | {(rd or 0) / 1e6:.1f} | {(wr or 0) / 1e6:.1f} | "
                f"{'-' if tbs is None else f'{tbs / 1e12:.2f}'} | "
                f"{'-' if tbs is None else f'{100 * tbs / HBM_ACHIEVABLE:.0f}%'} | "
                f"{'-' if fl is None else f'{fl / 1e9:.1f}'} | {'-' if tfs is None else f'{tfs / 1e12:.1f}'} | "
                f"{'-' if tfs is None else f'{100 * tfs / MFMA_PEAK:.1f}%'} |")

    hdr = ("| kernel class | ms/step | launches/step | MB read | MB written | TB/s | % of 6.3 TB/s | GFLOP (MFMA) | "
           "TFLOP/s | % of 2.5 PF |\n|---|---|---|---|---|---|---|---|---|---|")
    agg = defaultdict(lambda: [0.0, 0.0, 0.0, 0.0, 0.0, False, False])
    for r in rows:
        g = agg[r["cls"]]
        g[0] += r["ms"]
        g[1] += r["calls"]
        if r["rd"] is not None:
            g[2] += r["rd"]
            g[5] = True
        if r["wr"] is not None:
            g[3] += r["wr"]
        if r["fl"] is not None:
            g[4] += r["fl"]
            g[6] = True
    out = []
    tot = [0.0, 0.0, 0.0, 0.0, 0.0]
    out.append(f"Step window {window.get('ms_per_step', 0):.3f} ms, GPU busy {window.get('busy_ms_per_step', 0):.3f} ms.")
    out.append("")
    out.append("### By kernel class\n")
    out.append(hdr)
    for label, g in sorted(agg.items(), key=lambda kv: -kv[1][0]):
        out.append(line(label, g[0], g[1], g[2] if g[5] else None, g[3] if g[5] else None, g[4] if g[6] else None))
        for i in range(5):
            tot[i] += g[i]
    out.append(line("**total**", tot[0], tot[1], tot[2], tot[3], tot[4]))
    out.append("")
    out.append(f"### Top {a.top} kernels\n")
    out.append(hdr.replace("kernel class", "kernel"))
    for r in sorted(rows, key=lambda r: -r["ms"])[: a.top]:
        out.append(line(r["name"][:80], r["ms"], r["calls"], r["rd"], r["wr"], r["fl"]))
    text = "\n".join(out)
    print(text)
    if a.md:
        with open(a.md, "w") as fh:
            fh.write(text + "\n")


if __name__ == "__main__":
    main()
