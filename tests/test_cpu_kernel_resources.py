"""Register budget of the hot kernels, read from the built gfx950 code object (no GPU needed; tools/kernel_resources.py).

Guards the occupancy decisions DESIGN.md records: the kernels on the measured paths keep every value in registers
(no scratch: a spill turns the FP64 Brent loop into a memory-latency loop), and k_prep without the de novo
monomorphism path (MDN = false, every engine that does not form that product in k_prep) stays within the VGPR
budget that gives it the waves per SIMD its HBM-latency-bound chunk loop needs.
"""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "polymutt_amd", "lib", "libpolymutt.so")
sys.path.insert(0, os.path.join(ROOT, "tools"))

# headline quad plan, config-5 split plan, config-4 --denovo fused item, the posterior/finalize kernels
NO_SCRATCH = [
    "void k_brent<64, 16, 2, false, false, true, false, false, true, 0, 8>(DevArgs, int)",
    "void k_brent<128, 16, 2, false, false, false, true, false, false, 34, 8>(DevArgs, int)",
    "void k_brent<64, 1, 0, true, true, true, false, true, false, 1, 8>(DevArgs, int)",
    "void k_posterior_lean<true>(DevArgs)",
    "void k_posterior<true, false>(DevArgs)",
    "k_finalize(DevArgs)",
    "k_finalize_vcf(DevArgs)",
]
# k_prep<VEC, SERIAL, VC, MDN>: max VGPRs (512 / vgprs = waves per SIMD)
PREP_VGPR_MAX = {
    "void k_prep<8, false, true, false>(DevArgs, int)": 64,     # config 5 (vcf_mode): 8 waves
    "void k_prep<16, false, true, false>(DevArgs, int)": 96,
    "void k_prep<8, false, false, false>(DevArgs, int)": 128,   # headline (mono_dn == 2): 4 waves
    "void k_prep<4, false, false, false>(DevArgs, int)": 128,
}


def _resources():
    kr = pytest.importorskip("kernel_resources")
    if not os.path.exists(LIB):
        pytest.skip("libpolymutt.so not built (__graft_entry__.build())")
    if not os.path.exists(os.path.join(kr.LLVM, "llvm-readobj")) or not shutil.which("c++filt"):
        pytest.skip("llvm-readobj / c++filt not available")
    rows = [r for co in kr.code_objects(LIB) for r in kr.kernels(co)]
    names = subprocess.run(["c++filt"], input="\n".join(r.get("name", "?") for r in rows), capture_output=True,
                           text=True).stdout.splitlines()
    assert len(names) == len(rows)
    return {n.strip(): r for n, r in zip(names, rows)}


@pytest.fixture(scope="module")
def res():
    return _resources()


def test_hot_kernels_do_not_spill(res):
    for k in NO_SCRATCH:
        assert k in res, k
        assert int(res[k]["private_segment_fixed_size"]) == 0, (k, res[k])


def test_prep_without_denovo_mono_fits_its_wave_budget(res):
    for k, vmax in PREP_VGPR_MAX.items():
        assert k in res, k
        assert int(res[k]["vgpr_count"]) <= vmax, (k, res[k]["vgpr_count"], vmax)
    # the MDN variant keeps the ten-plane product (more registers): the split is what buys the occupancy
    assert int(res["void k_prep<8, false, false, true>(DevArgs, int)"]["vgpr_count"]) > \
        int(res["void k_prep<8, false, false, false>(DevArgs, int)"]["vgpr_count"])
