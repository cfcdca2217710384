"""TEST INFRASTRUCTURE ONLY — ctypes wrapper of oracle/_build/liboracle.so.

The CPU restatement of the reference hot path (oracle/mgp_oracle.c). Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may import this
module, and only as the checker; the product path (mgatk2_amd) never does.
"""

from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

from mgatk2_amd.engine import EngineConfig, EngineResult, batch_struct, mgp_batch, mgp_config, mgp_result, mgp_stats
from mgatk2_amd.synth import ReadSoA

ORACLE_SO = Path(__file__).resolve().parent / "_build" / "liboracle.so"
_lib = None


def _load():
    global _lib
    if _lib is None:
        if not ORACLE_SO.exists():
            from mgatk2_amd.build import build_oracle

            build_oracle()
        _lib = C.CDLL(str(ORACLE_SO))
        _lib.oracle_run.argtypes = [
            C.POINTER(mgp_config), C.POINTER(mgp_batch), C.POINTER(mgp_result),
            C.c_void_p, C.POINTER(C.c_int32),
        ]
        _lib.oracle_run.restype = C.c_int
    return _lib


class OracleError(RuntimeError):
    def __init__(self, code: int):
        self.code = code
        super().__init__(f"oracle_run failed with code {code}")


def oracle_run(cfg: EngineConfig, soa: ReadSoA, dense: bool = True) -> tuple[EngineResult, np.ndarray]:
    """Run the CPU restatement. Returns (result, first-seen barcode order)."""
    lib = _load()
    res = EngineResult.alloc(cfg.n_cells, cfg.mito_len, dense)
    st = mgp_stats()
    cres = res.to_c(st)
    ccfg = cfg.to_c()
    b = batch_struct(soa)
    order = np.full(max(cfg.n_cells, 1), -1, np.int32)
    n_order = C.c_int32()
    code = lib.oracle_run(C.byref(ccfg), C.byref(b), C.byref(cres), order.ctypes.data_as(C.c_void_p), C.byref(n_order))
    if code != 0:
        raise OracleError(code)
    res.stats = st.as_dict()
    return res, order[: n_order.value].copy()
