"""Split-K targets of the bf16 weight-gradient kernels, swept on the whole bench step.

    python scripts/sweep_splits.py WGRAD3_WG=256 IWGRAD_MINPIX=512 -- --steps 30 --no-fp32

Each ``NAME=value`` before ``--`` overrides ``garfield_amd.ops.grouped._NAME`` before the
engine is built; the arguments after ``--`` go to ``bench.py``. The split count trades
workgroups (occupancy) against fp32 slab traffic: every split writes a [G, cout, K] fp32
slab that the deferred reduction reads back.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    sets, rest = argv[:cut], argv[cut + 1:]
    from garfield_amd.ops import grouped

    for kv in sets:
        k, v = kv.split("=")
        name = "_" + k
        if not hasattr(grouped, name):
            raise SystemExit(f"no constant {name} in garfield_amd.ops.grouped")
        setattr(grouped, name, int(v))
    print("overrides:", {kv.split("=")[0]: int(kv.split("=")[1]) for kv in sets}, flush=True)
    import bench

    sys.argv = ["bench.py", *rest]
    bench.main()


if __name__ == "__main__":
    main()
