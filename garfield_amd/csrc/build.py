"""In-tree build of the native extension ``garfield_amd/_C*.so`` for gfx950.

Explicit ``hipcc --offload-arch=gfx950`` command lines (no hipify pass, no JIT
cache under ~/.cache): the shared object lands next to the package so it travels
with the repository snapshot to the GPU box.

Reference counterpart: the on-import JIT builder
``pytorch_impl/libs/native/__init__.py:19-156`` (cpp_extension.load, .deps graph,
NATIVE_OPT debug-by-default). Here the default is ``-O3``; ``GARFIELD_NATIVE_DEBUG=1``
gives ``-O0 -g``. Builds are incremental (object newer than its source and every
header) and parallel (``MAX_JOBS``).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shlex
import subprocess
import sys
import sysconfig
from pathlib import Path

CSRC = Path(__file__).resolve().parent
PKG = CSRC.parent
BUILD = PKG.parent / "build" / "garfield_native"
ARCH = os.environ.get("GARFIELD_OFFLOAD_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
HIPCC = str(ROCM / "bin" / "hipcc")

HIP_SOURCES = [
    "gar_gram.hip", "gar_combine.hip", "gar_coord.hip", "gar_flatten.hip",
    "gar_coord_m0.hip", "gar_coord_m1.hip", "gar_coord_m2.hip",
    "gar_coord_m3.hip", "gar_coord_m4.hip", "gar_coord_m5.hip",
    "bn_nhwc.hip", "im2col_nhwc.hip", "iconv_nhwc.hip", "gemm_nt.hip", "data_aug.hip", "gar_large.hip", "loss_xent.hip", "stream_signal.hip", "stem_nhwc.hip",
    "gar_layerwise.hip", "conv3x3_nhwc.hip", "conv_f32.hip", "sconv_nhwc.hip", "gar_tail_f32.hip",
]
TORCH_SOURCES = ["bindings.cpp", "mailbox.cpp", "rccl_direct.cpp"]   # need torch + HIP headers
PLAIN_SOURCES = ["threadpool.cpp", "gar_cpu.cpp"]  # plain C++17


def ext_path() -> Path:
    return PKG / ("_C" + sysconfig.get_config_var("EXT_SUFFIX"))


def _torch_flags():
    import torch
    from torch.utils import cpp_extension as ce

    incs = list(ce.include_paths())
    incs.append(sysconfig.get_paths()["include"])
    incs.append(str(ROCM / "include"))
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    defs = [
        "-DTORCH_EXTENSION_NAME=_C",
        "-DTORCH_API_INCLUDE_EXTENSION_H",
        f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DUSE_ROCM=1",
        "-D__HIP_PLATFORM_AMD__=1",
    ]
    try:
        defs += list(ce._get_pybind11_abi_build_flags())
    except Exception:  # older/newer torch: the ABI tags are optional
        pass
    libdir = str(Path(torch.__file__).parent / "lib")
    return incs, defs, libdir


def _opt_flags():
    if os.environ.get("GARFIELD_NATIVE_DEBUG", "0") == "1":
        return ["-O0", "-g"]
    return ["-O3", "-DNDEBUG"]


def _needs(obj: Path, src: Path) -> bool:
    if not obj.exists():
        return True
    t = obj.stat().st_mtime
    if src.stat().st_mtime > t:
        return True
    return any(h.stat().st_mtime > t for h in CSRC.glob("*.hpp"))


def _run(cmd, verbose):
    if verbose:
        print(" ".join(shlex.quote(c) for c in cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def sources_digest() -> str:
    """sha256 over every native source and header (name + bytes), the identity of a build."""
    import hashlib

    h = hashlib.sha256()
    for f in sorted([*CSRC.glob("*.hip"), *CSRC.glob("*.cpp"), *CSRC.glob("*.hpp")]):
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()


def manifest_path() -> Path:
    return PKG / "_C.build.json"


def build(verbose: bool = False, force: bool = False) -> Path:
    """Compile every source (parallel, incremental) and link ``_C``. Returns the .so path.
    Writes ``_C.build.json`` next to it: the sources' digest, how many translation units this
    call compiled, the target and the compiler, so a shipped .so can be matched to its sources."""
    incs, defs, libdir = _torch_flags()
    BUILD.mkdir(parents=True, exist_ok=True)
    opt = _opt_flags()
    inc_flags = [f"-I{i}" for i in incs] + [f"-I{CSRC}"]
    jobs = []
    for s in HIP_SOURCES:
        src, obj = CSRC / s, BUILD / (s + ".o")
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-std=c++17", "-fPIC", *opt, f"-I{CSRC}",
               "-D__HIP_PLATFORM_AMD__=1", "-c", str(src), "-o", str(obj)]
        jobs.append((obj, src, cmd))
    for s in TORCH_SOURCES:
        src, obj = CSRC / s, BUILD / (s + ".o")
        # host-only translation units: the HIP runtime API is plain C++ with __HIP_PLATFORM_AMD__
        cmd = ["g++", "-std=c++17", "-fPIC", *opt, *defs, *inc_flags, "-Wno-unused-result",
               "-Wno-deprecated-declarations", "-c", str(src), "-o", str(obj)]
        jobs.append((obj, src, cmd))
    for s in PLAIN_SOURCES:
        src, obj = CSRC / s, BUILD / (s + ".o")
        cmd = ["g++", "-std=c++17", "-fPIC", *opt, "-pthread", f"-I{CSRC}", "-c", str(src), "-o", str(obj)]
        jobs.append((obj, src, cmd))
    todo = [j for j in jobs if force or _needs(j[0], j[1])]
    nproc = max(1, min(int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=nproc) as ex:
            futs = [ex.submit(_run, cmd, verbose) for _, _, cmd in todo]
            for f in futs:
                f.result()
    out = ext_path()
    objs = [str(j[0]) for j in jobs]
    if force or todo or not out.exists() or any(Path(o).stat().st_mtime > out.stat().st_mtime for o in objs):
        link = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, "-o", str(out),
                f"-L{libdir}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip",
                f"-L{ROCM / 'lib'}", "-lamdhip64", "-pthread", "-ldl",
                f"-Wl,-rpath,{libdir}", f"-Wl,-rpath,{ROCM / 'lib'}"]
        _run(link, verbose)
    import json
    import time

    ver = subprocess.run([HIPCC, "--version"], capture_output=True, text=True).stdout.splitlines()
    manifest = {"sources_sha256": sources_digest(), "units": len(jobs), "compiled_this_call": len(todo),
                "linked_this_call": bool(force or todo) or not out.exists(), "arch": ARCH, "opt": opt,
                "compiler": next((v for v in ver if "version" in v.lower()), ""),
                "so_bytes": out.stat().st_size, "time": time.strftime("%Y-%m-%dT%H:%M:%S")}
    manifest_path().write_text(json.dumps(manifest, indent=1) + "\n")
    return out


def build_selftest(sanitizer: str = "thread", out_dir: Path | None = None) -> Path:
    """Host-only native self-test (thread pool, CPU GARs, mailbox) built with
    ``-fsanitize=<sanitizer>`` (thread | address | undefined). GPU sanitizers are not
    used: the sanitizer flags only ever reach host code (no HIP in this binary)."""
    out_dir = out_dir or BUILD
    out_dir.mkdir(parents=True, exist_ok=True)
    exe = out_dir / f"selftest_{sanitizer}"
    srcs = [CSRC / "selftest.cpp", CSRC / "threadpool.cpp", CSRC / "gar_cpu.cpp", CSRC / "mailbox.cpp"]
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={sanitizer}", "-fno-omit-frame-pointer",
           "-DGARFIELD_NO_TORCH", "-DGARFIELD_NO_HIP", f"-I{CSRC}", *map(str, srcs), "-o", str(exe), "-pthread"]
    _run(cmd, False)
    return exe


if __name__ == "__main__":
    p = build(verbose="-v" in sys.argv, force="--force" in sys.argv)
    print(p)
