"""polymutt_amd -- MI355X-native per-site family-likelihood engine for polyMutt.

The compute path is hand-written HIP for gfx950 behind a C ABI (include/polymutt_engine.h,
include/polymutt_host.h), built into ``polymutt_amd/lib/libpolymutt.so``; the ``polymutt`` CLI in
``polymutt_amd/bin`` is the drop-in replacement of the reference binary.  This Python module is a thin
ctypes binding for tests and the benchmark: it never computes anything itself and raises if the
native library is missing.
"""
from .engine import (  # noqa: F401
    LIB_PATH, BIN_PATH, load_library, Engine, Pedigree, GlfReader, Params, SiteResult, GenoCall, Counters,
    KernelStats, PedigreeStruct, NUM_PRODUCT, NUM_EXACT, NUM_POLY, PM_CHR_AUTO, PM_CHR_X, PM_CHR_Y, PM_CHR_MT, FAM_NUCLEAR, FAM_FOUNDERS,
    FAM_EXTENDED, synth_write_dataset, synth_block_host, planar, pedigree_from_arrays,
)
