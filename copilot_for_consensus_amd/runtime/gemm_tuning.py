"""Pre-tuned library GEMM selections (PyTorch TunableOp over hipBLASLt + rocBLAS solutions).

The plain projection GEMMs stay on the vendor libraries (hipBLASLt/rocBLAS); for the skinny
decode shapes (M = batch) the library heuristic picks poorly, so the best solution per shape was
measured on MI355X (scripts/bench_gemm.py with PYTORCH_TUNABLEOP_TUNING=1) and is shipped in
``tuning/gemm_mi355x.csv``.  At run time tuning is OFF: the file is only read, so there is no
search cost and hipGraph capture sees fixed kernels.  Shapes absent from the file use the
library default.
"""
from __future__ import annotations

import os
from pathlib import Path

DEFAULT_FILE = Path(__file__).resolve().parent / "tuning" / "gemm_mi355x.csv"
_enabled = False


def enable_tuned_gemms(path: str | os.PathLike | None = None) -> bool:
    global _enabled
    if _enabled or os.environ.get("CFC_TUNABLEOP", "1") == "0":
        return _enabled
    import torch
    if not torch.cuda.is_available():
        return False
    tun = torch.cuda.tunable
    p = str(path or DEFAULT_FILE)
    if not Path(p).exists():
        return False
    tun.enable(True)
    tun.tuning_enable(False)
    ok = bool(tun.read_file(p))
    _enabled = ok
    if not ok:
        tun.enable(False)
    return ok
