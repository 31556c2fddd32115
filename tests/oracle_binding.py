"""ctypes binding of the CPU oracle (oracle/pm_oracle.c) -- TEST INFRASTRUCTURE ONLY.

Used by tests/ as the parity checker of the HIP engine; shares the C structs of
include/polymutt_engine.h through polymutt_amd.engine's ctypes mirrors.
"""
import ctypes as C
import os

import numpy as np

from polymutt_amd.engine import (CALL_DTYPE, SITE_DTYPE, Counters, Params, PedigreeStruct)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "build", "libpm_oracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            import subprocess
            subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "build/libpm_oracle.so"], check=True)
        L = C.CDLL(ORACLE_SO)
        L.pmo_create.restype = C.c_void_p
        L.pmo_create.argtypes = [C.POINTER(PedigreeStruct), C.POINTER(Params)]
        L.pmo_destroy.argtypes = [C.c_void_p]
        L.pmo_begin_section.argtypes = [C.c_void_p, C.c_int32]
        L.pmo_poly_prior.restype = C.c_double
        L.pmo_poly_prior.argtypes = [C.c_void_p]
        L.pmo_site.restype = C.c_int
        L.pmo_site.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32, C.c_void_p, C.c_void_p]
        L.pmo_objective.restype = C.c_double
        L.pmo_objective.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_double, C.c_int32]
        L.pmo_poly_loglik.restype = C.c_double
        L.pmo_poly_loglik.argtypes = [C.c_void_p, C.c_void_p, C.c_int32, C.c_int32, C.c_int32,
                                      C.POINTER(C.c_double), C.POINTER(C.c_int32)]
        L.pmo_counters.argtypes = [C.c_void_p, C.POINTER(Counters)]
        _lib = L
    return _lib


class Oracle:
    def __init__(self, ped_struct, params):
        self.L = lib()
        self.ped = ped_struct
        self.params = params
        self.h = self.L.pmo_create(C.byref(ped_struct), C.byref(params))
        self.n_person = ped_struct.n_person

    def begin_section(self, chrom=0):
        self.L.pmo_begin_section(self.h, chrom)

    def run(self, pl, dm, ref):
        """Same contract as polymutt_amd.Engine.run: (results[n], calls[rows, n_person])."""
        n = len(ref)
        pl = np.ascontiguousarray(pl, dtype=np.uint8).reshape(n, self.n_person, 10)
        dm = np.ascontiguousarray(dm, dtype=np.uint32).reshape(n, self.n_person)
        res = np.zeros(n, dtype=SITE_DTYPE)
        calls = np.zeros((n, self.n_person), dtype=CALL_DTYPE)
        rows = 0
        for i in range(n):
            rc = self.L.pmo_site(self.h, pl[i].ctypes.data, dm[i].ctypes.data, int(ref[i]),
                                 res[i:i + 1].ctypes.data, calls[rows].ctypes.data)
            if rc != 0:
                raise FloatingPointError("ScalarMinimizer::Brent got stuck")
            if res[i]["emit"] == 1:   # rows for written records only (emit 2 = suppressed de novo record)
                res[i]["call_row"] = rows
                rows += 1
            else:
                res[i]["call_row"] = -1
        return res, calls[:rows]

    def counters(self):
        c = Counters()
        self.L.pmo_counters(self.h, C.byref(c))
        return c

    def objective(self, pl_site, a1, a2, freq, denovo=0):
        pl_site = np.ascontiguousarray(pl_site, dtype=np.uint8)
        return self.L.pmo_objective(self.h, pl_site.ctypes.data, a1, a2, freq, denovo)

    def __del__(self):
        if getattr(self, "h", None):
            self.L.pmo_destroy(self.h)
            self.h = None
