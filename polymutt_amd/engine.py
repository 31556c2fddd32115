"""ctypes binding of libpolymutt.so (include/polymutt_engine.h + include/polymutt_host.h).

Mirrors the reference's per-site call surface (FamilyLikelihoodSeq / NucFamGenotypeLikelihood, see
SURVEY.md section 8(b)) at batch granularity: ``Engine.run`` evaluates a batch of sites the way one
iteration of src/main.cpp:327-589 evaluates one site.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("POLYMUTT_LIB") or os.path.join(_HERE, "lib", "libpolymutt.so")   # override: experiments
BIN_PATH = os.path.join(_HERE, "bin", "polymutt")

PM_CHR_AUTO, PM_CHR_X, PM_CHR_Y, PM_CHR_MT = 0, 1, 2, 3
FAM_NUCLEAR, FAM_FOUNDERS, FAM_EXTENDED = 0, 1, 2
PM_EBRENT = -4


class BrentStuck(FloatingPointError):
    """PM_EBRENT: a site's Brent maximisation hit ITMAX ("ScalarMinimizer::Brent got stuck", core/MathGold.cpp:98,175).
    ``site`` = the batch index of the first such site; ``results`` / ``calls`` = the batch's results and the genotype
    rows of the sites before it (complete, as the reference had written them before exiting)."""

    def __init__(self, site, results=None, calls=None):
        super().__init__("ScalarMinimizer::Brent got stuck")
        self.site, self.results, self.calls = site, results, calls

i32, i64, u64, f64, i8, i16 = C.c_int32, C.c_int64, C.c_uint64, C.c_double, C.c_int8, C.c_int16
P = C.POINTER


class PeelStep(C.Structure):
    _fields_ = [("type", i32), ("from0", i32), ("from1", i32), ("to0", i32), ("to1", i32)]


class PedigreeStruct(C.Structure):
    _fields_ = [("n_fam", i32), ("n_person", i32), ("fam_start", P(i32)), ("fam_founders", P(i32)),
                ("fam_kind", P(i32)), ("sex", P(i8)), ("is_founder", P(i8)), ("father", P(i32)),
                ("mother", P(i32)), ("peel_start", P(i32)), ("steps", P(PeelStep)), ("n_founders", i32),
                ("male_founders", i32), ("female_founders", i32)]


NUM_PRODUCT, NUM_EXACT, NUM_POLY = 0, 1, 2   # pm_numerics


class Params(C.Structure):
    _fields_ = [("theta", f64), ("poly_tstv", f64), ("precision", f64), ("posterior", f64),
                ("min_total_depth", i32), ("max_total_depth", i32), ("min_ps", f64), ("min_map_quality", i32),
                ("denovo", i32), ("denovo_mut_rate", f64), ("denovo_tstv", f64), ("denovo_min_llr", f64),
                ("force_call", i32), ("all_sites", i32), ("quick_call", i32), ("numerics", i32), ("vcf_mode", i32)]

    @classmethod
    def defaults(cls, **kw):
        """Defaults of src/main.cpp:59-85."""
        p = cls(theta=0.001, poly_tstv=2.0, precision=0.0001, posterior=0.5, min_total_depth=0, max_total_depth=0,
                min_ps=0.0, min_map_quality=0, denovo=0, denovo_mut_rate=1.5e-8, denovo_tstv=2.0,
                denovo_min_llr=0.01, force_call=0, all_sites=0, quick_call=0, numerics=NUM_POLY, vcf_mode=0)
        for k, v in kw.items():
            setattr(p, k, v)
        return p


class SiteResult(C.Structure):
    _fields_ = [("status", i32), ("n_cfg", i32), ("maxidx", i32), ("emit", i32), ("total_depth", i32),
                ("num_samp_with_data", i32), ("avg_map_qual", f64), ("perc_samp_with_data", f64),
                ("var_post_prob", f64), ("poly_qual", f64), ("varllk", f64 * 7), ("varfreq", f64 * 7),
                ("af", f64), ("ab", f64), ("denovo_lr", f64), ("evals", i32 * 7), ("allele1", i32),
                ("allele2", i32), ("is_mono", i32), ("denovo_mono", i32), ("call_row", i32)]


class GenoCall(C.Structure):
    _fields_ = [("dosage", f64), ("best", i16), ("gq", i16), ("label", i8), ("_pad", i8 * 3)]


class Counters(C.Structure):
    _fields_ = [("ref_base_counts", i64 * 5), ("min_total_depth_filter", i64), ("max_total_depth_filter", i64),
                ("min_ps_filter", i64), ("min_map_qual_filter", i64), ("homo_ref", i64), ("transitions", i64),
                ("transversions", i64), ("tstvs1", i64), ("tstvs2", i64), ("tvs1tvs2", i64), ("nocall", i64)]

    def as_array(self):
        return np.array(list(self.ref_base_counts) + [getattr(self, n) for n, _ in self._fields_[1:]], dtype=np.int64)


class KernelStats(C.Structure):
    _fields_ = [("launches", i64), ("kernel_ms", f64), ("evals", i64), ("fam_evals", i64), ("items", i64),
                ("sites", i64), ("site_visits", i64), ("hoist_wave_ns", i64), ("eval_wave_ns", i64),
                ("timed_items", i64), ("es_hoist_launches", i64), ("es_hoist_ms", f64), ("es_hoist_ops", f64)]


SITE_DTYPE = np.dtype([
    ("status", "<i4"), ("n_cfg", "<i4"), ("maxidx", "<i4"), ("emit", "<i4"), ("total_depth", "<i4"),
    ("num_samp_with_data", "<i4"), ("avg_map_qual", "<f8"), ("perc_samp_with_data", "<f8"),
    ("var_post_prob", "<f8"), ("poly_qual", "<f8"), ("varllk", "<f8", (7,)), ("varfreq", "<f8", (7,)),
    ("af", "<f8"), ("ab", "<f8"), ("denovo_lr", "<f8"), ("evals", "<i4", (7,)), ("allele1", "<i4"),
    ("allele2", "<i4"), ("is_mono", "<i4"), ("denovo_mono", "<i4"), ("call_row", "<i4")])
CALL_DTYPE = np.dtype([("dosage", "<f8"), ("best", "<i2"), ("gq", "<i2"), ("label", "i1"), ("_pad", "i1", (3,))])
VCF_CALL_DTYPE = np.dtype([("best", "i1"), ("gq", "i1"), ("label", "i1"), ("pad", "i1")])   # pm_vcf_call
assert SITE_DTYPE.itemsize == C.sizeof(SiteResult) == 240, SITE_DTYPE.itemsize
assert CALL_DTYPE.itemsize == C.sizeof(GenoCall) == 16

_lib = None

EXPORTS = {
    # include/polymutt_engine.h
    "pm_engine_create": (i32, [P(PedigreeStruct), P(Params), i32, i32, P(C.c_void_p)]),
    "pm_engine_destroy": (None, [C.c_void_p]),
    "pm_engine_plan": (i32, [C.c_void_p, P(i32), P(i32)]),
    "pm_engine_set_posterior_carry": (i32, [C.c_void_p, i32]),
    "pm_engine_begin_section": (i32, [C.c_void_p, i32]),
    "pm_engine_run": (i32, [C.c_void_p, i32, C.c_void_p, C.c_void_p, C.c_void_p, i32, C.c_void_p, C.c_void_p, P(i32)]),
    "pm_engine_run_vcf": (i32, [C.c_void_p, i32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, P(i32)]),
    "pm_engine_run_device": (i32, [C.c_void_p, i32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "pm_engine_sync": (i32, [C.c_void_p]),
    "pm_engine_submit": (i32, [C.c_void_p, i32, C.c_void_p, C.c_void_p, C.c_void_p]),
    "pm_engine_collect": (i32, [C.c_void_p, C.c_void_p, C.c_void_p, P(i32)]),
    "pm_engine_stuck_site": (i32, [C.c_void_p, P(i32)]),
    "pm_host_alloc": (i32, [u64, P(C.c_void_p)]),
    "pm_host_free": (i32, [C.c_void_p]),
    "pm_engine_to_planar": (i32, [C.c_void_p, i32, C.c_void_p, C.c_void_p]),
    "pm_engine_counters": (i32, [C.c_void_p, P(Counters)]),
    "pm_engine_synth": (i32, [C.c_void_p, i32, u64, u64, C.c_void_p, C.c_void_p, C.c_void_p]),
    "pm_device_alloc": (i32, [C.c_void_p, u64, P(C.c_void_p)]),
    "pm_device_free": (i32, [C.c_void_p, C.c_void_p]),
    "pm_copy_to_host": (i32, [C.c_void_p, C.c_void_p, C.c_void_p, u64]),
    "pm_copy_to_device": (i32, [C.c_void_p, C.c_void_p, C.c_void_p, u64]),
    "pm_engine_kernel_stats": (i32, [C.c_void_p, P(KernelStats), i32]),
    "pm_last_error": (C.c_char_p, []),
    "pm_abi_version": (i32, []),
    # include/polymutt_host.h
    "pmh_pedigree_load": (C.c_void_p, [C.c_char_p, C.c_char_p]),
    "pmh_pedigree_view": (i32, [C.c_void_p, P(PedigreeStruct)]),
    "pmh_pedigree_pid": (C.c_char_p, [C.c_void_p, i32]),
    "pmh_pedigree_famid": (C.c_char_p, [C.c_void_p, i32]),
    "pmh_pedigree_is_nuclear": (i32, [C.c_void_p, i32]),
    "pmh_pedigree_free": (None, [C.c_void_p]),
    "pmh_glf_open": (C.c_void_p, [C.c_void_p, C.c_char_p]),
    "pmh_glf_next_section": (i32, [C.c_void_p, C.c_char_p, i32, P(i32)]),
    "pmh_glf_read_sites": (i32, [C.c_void_p, i32, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "pmh_glf_close": (None, [C.c_void_p]),
    "pmh_synth_write_dataset": (i32, [C.c_char_p, C.c_char_p, i32, i32, u64]),
    "pmh_run_polymutt": (i32, [i32, P(C.c_char_p), i32, i32, i32, C.c_void_p, C.c_void_p]),   # see launch.py
    "pmh_synth_block": (i32, [P(PedigreeStruct), i32, u64, u64, C.c_void_p, C.c_void_p, C.c_void_p]),
}


def load_library(path=LIB_PATH):
    """Load libpolymutt.so and declare every exported symbol (fails loudly if missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"native engine library not built: {path} (run __graft_entry__.build())")
    lib = C.CDLL(path)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _err(lib):
    return lib.pm_last_error().decode(errors="replace")


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p)


class Pedigree:
    """Pedigree loaded by the native Merlin .dat/.ped loader (polyMutt ordering)."""

    def __init__(self, dat_file, ped_file):
        self.lib = load_library()
        self.h = self.lib.pmh_pedigree_load(dat_file.encode(), ped_file.encode())
        if not self.h:
            raise RuntimeError(_err(self.lib))
        self.view = PedigreeStruct()
        assert self.lib.pmh_pedigree_view(self.h, C.byref(self.view)) == 0

    @property
    def n_person(self):
        return self.view.n_person

    @property
    def n_fam(self):
        return self.view.n_fam

    def pids(self):
        return [self.lib.pmh_pedigree_pid(self.h, i).decode() for i in range(self.n_person)]

    def fam_start(self):
        return np.ctypeslib.as_array(self.view.fam_start, shape=(self.n_fam + 1,)).copy()

    def fam_kind(self):
        return np.ctypeslib.as_array(self.view.fam_kind, shape=(self.n_fam,)).copy()

    def sex(self):
        return np.ctypeslib.as_array(self.view.sex, shape=(self.n_person,)).copy()

    def is_nuclear(self, f):
        return bool(self.lib.pmh_pedigree_is_nuclear(self.h, f))

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.pmh_pedigree_free(self.h)
            self.h = None


def pedigree_from_arrays(fam_sizes, fam_founders, fam_kind, sex, is_founder, father, mother, n_founders=None,
                         male_founders=None, female_founders=None):
    """Build a PedigreeStruct from numpy arrays (kept alive on the returned object)."""
    keep = {}

    def arr(name, a, dt):
        keep[name] = np.ascontiguousarray(a, dtype=dt)
        return keep[name].ctypes.data_as(P({np.int32: i32, np.int8: i8}[dt]))

    fs = np.concatenate([[0], np.cumsum(fam_sizes)]).astype(np.int32)
    ps = PedigreeStruct()
    ps.n_fam = len(fam_sizes)
    ps.n_person = int(fs[-1])
    ps.fam_start = arr("fs", fs, np.int32)
    ps.fam_founders = arr("ff", fam_founders, np.int32)
    ps.fam_kind = arr("fk", fam_kind, np.int32)
    ps.sex = arr("sex", sex, np.int8)
    ps.is_founder = arr("isf", is_founder, np.int8)
    ps.father = arr("fa", father, np.int32)
    ps.mother = arr("mo", mother, np.int32)
    ps.peel_start = arr("pst", np.zeros(ps.n_fam + 1), np.int32)
    ps.steps = None
    isf = np.asarray(is_founder, dtype=bool)
    sx = np.asarray(sex)
    ps.n_founders = int(isf.sum()) if n_founders is None else n_founders
    ps.male_founders = int((isf & (sx == 1)).sum()) if male_founders is None else male_founders
    ps.female_founders = int((isf & (sx == 2)).sum()) if female_founders is None else female_founders
    ps._keep = keep
    return ps


class Engine:
    """One pm_engine on one HIP device.  No CPU fallback: construction fails without a GPU."""

    def __init__(self, ped_struct, params=None, device=0, max_batch=4096):
        self.lib = load_library()
        self.ped = ped_struct
        self.params = params or Params.defaults()
        self.n_person = ped_struct.n_person
        self.max_batch = max_batch
        h = C.c_void_p()
        rc = self.lib.pm_engine_create(C.byref(ped_struct), C.byref(self.params), device, max_batch, C.byref(h))
        if rc != 0:
            raise RuntimeError(f"pm_engine_create failed ({rc}): {_err(self.lib)}")
        self.h = h

    def begin_section(self, chrom=PM_CHR_AUTO):
        self._check(self.lib.pm_engine_begin_section(self.h, chrom))

    def run(self, pl, dm, ref):
        """Evaluate a batch of sites (host arrays).  Returns (results[n] structured array, calls[rows, n_person])."""
        n = len(ref)
        pl = np.ascontiguousarray(pl, dtype=np.uint8).reshape(n, self.n_person, 10)
        dm = np.ascontiguousarray(dm, dtype=np.uint32).reshape(n, self.n_person)
        ref = np.ascontiguousarray(ref, dtype=np.uint8)
        res = np.zeros(n, dtype=SITE_DTYPE)
        calls = np.zeros((n, self.n_person), dtype=CALL_DTYPE)
        rows = i32(0)
        self._check(self.lib.pm_engine_run(self.h, n, _ptr(pl), _ptr(dm), _ptr(ref), 0, _ptr(res), _ptr(calls),
                                           C.byref(rows)), res, calls, rows)
        return res, calls[: rows.value]

    def run_vcf(self, pl, ref):
        """pm_engine_run_vcf (vcf_mode engines): (results[n], calls[rows, n_person] of VCF_CALL_DTYPE, 4 B each)."""
        n = len(ref)
        pl = np.ascontiguousarray(pl, dtype=np.uint8).reshape(n, self.n_person, 10)
        ref = np.ascontiguousarray(ref, dtype=np.uint8)
        res = np.zeros(n, dtype=SITE_DTYPE)
        calls = np.zeros((n, self.n_person), dtype=VCF_CALL_DTYPE)
        rows = i32(0)
        self._check(self.lib.pm_engine_run_vcf(self.h, n, _ptr(pl), _ptr(ref), _ptr(res), _ptr(calls), C.byref(rows)),
                    res, calls, rows)
        return res, calls[: rows.value]

    def submit(self, pl, dm, ref):
        """pm_engine_submit: queue a batch of host arrays (kept referenced until collect()); returns at once."""
        n = len(ref)
        self._pending = (np.ascontiguousarray(pl, dtype=np.uint8).reshape(n, self.n_person, 10),
                         np.ascontiguousarray(dm, dtype=np.uint32).reshape(n, self.n_person),
                         np.ascontiguousarray(ref, dtype=np.uint8))
        pl, dm, ref = self._pending
        self._check(self.lib.pm_engine_submit(self.h, n, _ptr(pl), _ptr(dm), _ptr(ref)))

    def collect(self):
        """pm_engine_collect: wait for the submitted batch; (results[n], calls[rows, n_person]) as run() returns."""
        n = len(self._pending[2])
        res = np.zeros(n, dtype=SITE_DTYPE)
        calls = np.zeros((n, self.n_person), dtype=CALL_DTYPE)
        rows = i32(0)
        self._pending = None
        self._check(self.lib.pm_engine_collect(self.h, _ptr(res), _ptr(calls), C.byref(rows)), res, calls, rows)
        return res, calls[: rows.value]

    def run_device(self, n, d_pl, d_dm, d_ref, d_res=None, d_calls=None):
        """d_pl in the engine's genotype-planar layout [n][10][n_person] (pm_engine_synth, to_planar)."""
        self._check(self.lib.pm_engine_run_device(self.h, n, d_pl, d_dm, d_ref, d_res, d_calls))

    def to_planar(self, n, d_src, d_dst):
        """Person-major device block [n][n_person][10] -> genotype-planar [n][10][n_person]."""
        self._check(self.lib.pm_engine_to_planar(self.h, n, d_src, d_dst))

    def sync(self):
        self._check(self.lib.pm_engine_sync(self.h))

    def counters(self):
        c = Counters()
        self._check(self.lib.pm_engine_counters(self.h, C.byref(c)))
        return c

    def alloc(self, nbytes):
        p = C.c_void_p()
        self._check(self.lib.pm_device_alloc(self.h, nbytes, C.byref(p)))
        return p

    def free(self, p):
        self._check(self.lib.pm_device_free(self.h, p))

    def to_device(self, d_dst, src, nbytes):
        src = np.ascontiguousarray(src)
        self._check(self.lib.pm_copy_to_device(self.h, d_dst, _ptr(src), nbytes))

    def to_host(self, dst, d_src, nbytes):
        self._check(self.lib.pm_copy_to_host(self.h, _ptr(dst), d_src, nbytes))

    def synth(self, n, seed, site_offset, d_pl, d_dm, d_ref):
        self._check(self.lib.pm_engine_synth(self.h, n, seed, site_offset, d_pl, d_dm, d_ref))

    def set_posterior_carry(self, seen):
        self._check(self.lib.pm_engine_set_posterior_carry(self.h, 1 if seen else 0))

    def plan(self):
        """(threads per Brent item, family slots per lane) of the engine's lane plan."""
        t, s = i32(0), i32(0)
        self._check(self.lib.pm_engine_plan(self.h, C.byref(t), C.byref(s)))
        return t.value, s.value

    def kernel_stats(self, reset=False):
        s = KernelStats()
        self._check(self.lib.pm_engine_kernel_stats(self.h, C.byref(s), 1 if reset else 0))
        return s

    def stuck_site(self):
        """pm_engine_stuck_site: the first site of the last finished batch whose Brent hit ITMAX (-1: none)."""
        k = i32(0)
        self._check(self.lib.pm_engine_stuck_site(self.h, C.byref(k)))
        return k.value

    def _check(self, rc, res=None, calls=None, rows=None):
        if rc == PM_EBRENT:
            raise BrentStuck(self.stuck_site(), res, None if calls is None else calls[: rows.value])
        if rc != 0:
            raise RuntimeError(f"engine call failed ({rc}): {_err(self.lib)}")

    def close(self):
        if getattr(self, "h", None):
            self.lib.pm_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()


class GlfReader:
    """Dense per-site blocks from a GLF dataset through the native reader (PedigreeGLF semantics)."""

    def __init__(self, pedigree, glf_index_file):
        self.lib = load_library()
        self.ped = pedigree
        self.h = self.lib.pmh_glf_open(pedigree.h, glf_index_file.encode())
        if not self.h:
            raise RuntimeError(_err(self.lib))

    def sections(self):
        buf = C.create_string_buffer(4096)
        mp = i32(0)
        while self.lib.pmh_glf_next_section(self.h, buf, 4096, C.byref(mp)) == 1:
            yield buf.value.decode(), mp.value

    def read(self, max_sites):
        npers = self.ped.n_person
        pos = np.zeros(max_sites, np.int32)
        ref = np.zeros(max_sites, np.uint8)
        pl = np.zeros((max_sites, npers, 10), np.uint8)
        dm = np.zeros((max_sites, npers), np.uint32)
        n = self.lib.pmh_glf_read_sites(self.h, max_sites, _ptr(pos), _ptr(ref), _ptr(pl), _ptr(dm))
        if n < 0:
            raise RuntimeError(_err(self.lib))
        return pos[:n], ref[:n], pl[:n], dm[:n]

    def close(self):
        if getattr(self, "h", None):
            self.lib.pmh_glf_close(self.h)
            self.h = None

    def __del__(self):
        self.close()


def synth_write_dataset(directory, shape, n_fam, n_sites, seed):
    lib = load_library()
    if lib.pmh_synth_write_dataset(directory.encode(), shape.encode(), n_fam, n_sites, seed) != 0:
        raise RuntimeError(_err(lib))


def planar(pl):
    """Person-major [n][n_person][10] -> the engine's genotype-planar [n][10][n_person] (numpy)."""
    n = pl.shape[0]
    return np.ascontiguousarray(np.asarray(pl).reshape(n, -1, 10).transpose(0, 2, 1))


def synth_block_host(ped_struct, n, seed, site_offset=0):
    """Host-side generation of the sites pm_engine_synth writes on the device (same RNG), as person-major
    GLF records [n][n_person][10] (pm_engine_run's layout; planar(pl) gives the device layout)."""
    lib = load_library()
    npers = ped_struct.n_person
    pl = np.zeros((n, npers, 10), np.uint8)
    dm = np.zeros((n, npers), np.uint32)
    ref = np.zeros(n, np.uint8)
    if lib.pmh_synth_block(C.byref(ped_struct), n, seed, site_offset, _ptr(pl), _ptr(dm), _ptr(ref)) != 0:
        raise RuntimeError(_err(lib))
    return pl, dm, ref
