"""A/B of a kernel-form experiment switch (bindings.cpp ``_set_kernel_variant``) on a bench.py run:

    python scripts/ab_variant.py NAME VALUE [bench.py args ...]

sets the switch, then runs bench.py's main() in this process (one JSON line, as bench.py)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    name, val = sys.argv[1], int(sys.argv[2])
    sys.argv = [os.path.join(ROOT, "bench.py"), *sys.argv[3:]]
    from garfield_amd import _native

    _native.native()._set_kernel_variant(name, val)
    import bench

    bench.main()


if __name__ == "__main__":
    main()
