"""In-tree build of madnn's native code (gfx950 HIP kernels + C++ runtime).

Produces two shared objects next to this file:

* ``_madnn_kernels.so`` — the hand-written CDNA4 kernels (bucket pack/unpack,
  fused SGD/Adam, LayerNorm/RMSNorm) registered as ``torch.ops.madnn.*``.
* ``_madnn_runtime.so`` — host-only C++ runtime pieces (stage partitioner,
  bucket planner, collective-order hashing) exposed through a C ABI and
  loaded with ``ctypes``.

hipcc is driven directly (``--offload-arch=gfx950``), with no hipify step and
no JIT cache outside the repository, so the built ``.so`` files travel with
the repo snapshot to the GPU box.  ``python -m madnn.ops.build`` rebuilds
whatever is stale.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import json
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
BUILD = HERE / "_build"
KERNELS_SO = HERE / "_madnn_kernels.so"
RUNTIME_SO = HERE / "_madnn_runtime.so"
# source digests the shipped .so files were linked from (stale-binary guard, see stale_sources)
MANIFEST = HERE / "_madnn_build_manifest.json"

ARCH = os.environ.get("MADNN_OFFLOAD_ARCH", "gfx950")
KERNEL_SOURCES = ["bucket.hip", "optim.hip", "norm.hip", "bn.hip", "xent.hip", "pool.hip", "attn.hip", "conv.hip",
                  "stem.hip", "bias.hip", "gemm.hip", "gemmp.hip", "conv3.hip", "xgmi.hip", "probe.hip", "glue.hip",
                  "binding.cpp", "lt.cpp"]
RUNTIME_SOURCES = ["runtime.cpp"]
# per-source extra flags: MFMA kernels keep their accumulators in the (unified) VGPR file
# instead of AGPRs, which removes a v_accvgpr_read/write around every softmax element
EXTRA_FLAGS = {"attn.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1", "-fno-slp-vectorize"]}


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found: madnn's gfx950 kernels need ROCm's hipcc")


def _torch_paths():
    import torch

    root = Path(torch.__file__).resolve().parent
    inc = [root / "include", root / "include" / "torch" / "csrc" / "api" / "include"]
    return root, inc, root / "lib", int(torch._C._GLIBCXX_USE_CXX11_ABI)


def _flags_kernels():
    _, inc, _, abi = _torch_paths()
    flags = [
        "-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-fno-gpu-rdc",
        "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", "-DHIPBLAS_V2",
        "-DHIP_ENABLE_WARP_SYNC_BUILTINS=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-DTORCH_EXTENSION_NAME=_madnn_kernels", "-Wno-unused-result",
    ]
    flags += [f"-I{p}" for p in inc]
    flags += [f"-I{sysconfig.get_paths()['include']}", f"-I{CSRC}"]
    return flags


def _digest(paths, flags) -> str:
    h = hashlib.sha256()
    for p in paths:
        h.update(Path(p).read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()[:16]


def source_digests(csrc: Path = CSRC) -> dict:
    """sha256[:16] of every native source and header (what a built .so depends on)."""
    out = {}
    for name in KERNEL_SOURCES + RUNTIME_SOURCES + sorted(p.name for p in csrc.glob("*.h")):
        f = csrc / name
        if f.exists():
            out[name] = hashlib.sha256(f.read_bytes()).hexdigest()[:16]
    return out


def write_manifest(csrc: Path = CSRC, path: Path = MANIFEST) -> None:
    path.write_text(json.dumps({"arch": ARCH, "sources": source_digests(csrc)}, indent=1, sort_keys=True))


def stale_sources(csrc: Path = CSRC, path: Path = MANIFEST) -> list:
    """Sources whose current content differs from what the shipped .so was built from
    (every source if there is no manifest).  Empty list = the binary matches the tree."""
    cur = source_digests(csrc)
    try:
        built = json.loads(Path(path).read_text())
    except (OSError, ValueError):
        return sorted(cur)
    if built.get("arch") != ARCH:
        return sorted(cur)
    old = built.get("sources", {})
    return sorted(n for n in set(cur) | set(old) if cur.get(n) != old.get(n))


def _compile(src: Path, obj: Path, cmd_prefix, flags, verbose: bool):
    headers = sorted(CSRC.glob("*.h"))
    stamp = obj.with_suffix(".stamp")
    dig = _digest([src, *headers], flags)
    if obj.exists() and stamp.exists() and stamp.read_text() == dig:
        return False
    cmd = [*cmd_prefix, *flags, "-c", str(src), "-o", str(obj)]
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"compile failed: {src.name}\n{res.stdout}\n{res.stderr}")
    stamp.write_text(dig)
    return True


def build(verbose: bool = False, jobs: int | None = None, force: bool = False) -> dict:
    """Compile every native source for gfx950 and link the two shared objects."""
    BUILD.mkdir(exist_ok=True)
    if force:
        for p in BUILD.glob("*"):
            p.unlink()
    hipcc = _hipcc()
    kflags = _flags_kernels()
    rflags = ["-O3", "-std=c++17", "-fPIC", "-Wall", f"-I{CSRC}"]
    jobs = jobs or min(8, os.cpu_count() or 4)
    changed = False
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = []
        for s in KERNEL_SOURCES:
            futs.append(ex.submit(_compile, CSRC / s, BUILD / (s + ".o"), [hipcc],
                                  kflags + EXTRA_FLAGS.get(s, []), verbose))
        for s in RUNTIME_SOURCES:
            futs.append(ex.submit(_compile, CSRC / s, BUILD / (s + ".o"), ["g++"], rflags, verbose))
        for f in futs:
            changed |= f.result()

    troot, _, tlib, _ = _torch_paths()
    if changed or not KERNELS_SO.exists():
        objs = [str(BUILD / (s + ".o")) for s in KERNEL_SOURCES]
        cmd = [hipcc, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", str(KERNELS_SO),
               f"-L{tlib}", "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_hip", "-lhipblaslt",
               f"-Wl,-rpath,{tlib}"]
        if verbose:
            print(" ".join(cmd), flush=True)
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed: {KERNELS_SO.name}\n{res.stdout}\n{res.stderr}")
    if changed or not RUNTIME_SO.exists():
        objs = [str(BUILD / (s + ".o")) for s in RUNTIME_SOURCES]
        cmd = ["g++", "-shared", "-fPIC", *objs, "-o", str(RUNTIME_SO)]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed: {RUNTIME_SO.name}\n{res.stdout}\n{res.stderr}")
    if changed or not MANIFEST.exists() or stale_sources():
        write_manifest()
    return {"kernels": str(KERNELS_SO), "runtime": str(RUNTIME_SO), "arch": ARCH}


if __name__ == "__main__":
    out = build(verbose="-v" in sys.argv, force="--force" in sys.argv)
    print(out)
