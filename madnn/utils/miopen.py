"""MIOpen convolution-solver database handling.

With ``torch.backends.cudnn.benchmark = True`` PyTorch-ROCm runs MIOpen's *find*
for every new convolution shape: it compiles and times each applicable solver
and keeps the fastest (minutes for ResNet-50, most of it in the naive reference
solvers).  MIOpen records the winners in a text *user find-db*
(``<arch>.HIP.<version>.ufdb.txt``) and tuned solver parameters in a *user
perf-db* (``.udb.txt``).  Immediate mode (``benchmark = False``) also consults
the find-db before falling back to its heuristic, so with the db present both
modes start in about a second and pick the measured-fastest kernels:
ResNet-50 bs512 on one MI355X goes from 8.8k img/s (heuristic choice) to
9.8k img/s (profiles/r1_bench_resnet50_dp1_finddb.log).

madnn ships the dbs measured on MI355X (gfx950) under ``madnn/tuning/miopen/``
and seeds a per-process copy before the first convolution (``madnn.init`` does
this), so every rank starts from the tuned state and may add new shapes
without racing the others on one file.
"""
from __future__ import annotations

import atexit
import os
import shutil
import tempfile
from pathlib import Path
from typing import Optional

SHIPPED_DB = Path(__file__).resolve().parent.parent / "tuning" / "miopen"


def setup_find_db(src: Optional[os.PathLike] = None, workdir: Optional[os.PathLike] = None) -> str:
    """Point ``MIOPEN_USER_DB_PATH`` at a writable copy of the shipped db (no-op when the
    variable is already set).  Must run before the process's first convolution."""
    cur = os.environ.get("MIOPEN_USER_DB_PATH")
    if cur:
        return cur
    src = Path(src) if src else SHIPPED_DB
    if workdir:
        work = Path(workdir)
    else:
        work = Path(tempfile.mkdtemp(prefix="madnn_miopen_"))
        atexit.register(shutil.rmtree, work, True)
    work.mkdir(parents=True, exist_ok=True)
    if src.is_dir():
        for f in src.iterdir():
            if f.is_file() and (f.name.endswith(".txt") or f.name.endswith(".db")):
                shutil.copy2(f, work / f.name)
    os.environ["MIOPEN_USER_DB_PATH"] = str(work)
    return str(work)
