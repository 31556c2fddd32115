"""GPU parity tests: the HIP engine (through the C ABI) against the CPU oracle and the reference's
golden VCFs.  Marked gpu; run on an MI355X with `pytest -m gpu`."""
import os
import subprocess
import sys

import ctypes as C

import numpy as np
import pytest

import polymutt_amd as pm
from conftest import EXAMPLE, ROOT
from oracle_binding import Oracle
from parity import compare_results

pytestmark = pytest.mark.gpu


def _read_all(ped, gif_dir, gif="test.gif"):
    cwd = os.getcwd()
    os.chdir(gif_dir)
    try:
        rd = pm.GlfReader(ped, gif)
    finally:
        os.chdir(cwd)
    out = []
    for label, _ in rd.sections():
        pos, ref, pl, dm = rd.read(200000)
        out.append((label, pos, ref, pl, dm))
    return out


def _run_both(ped, params, sections, batch=4096, chrom_of=lambda lab: pm.PM_CHR_AUTO):
    eng = pm.Engine(ped.view, params, max_batch=batch)
    ora = Oracle(ped.view, params)
    stats = []
    for label, pos, ref, pl, dm in sections:
        ch = chrom_of(label)
        eng.begin_section(ch)
        ora.begin_section(ch)
        for s in range(0, len(ref), batch):
            e, ec = eng.run(pl[s:s + batch], dm[s:s + batch], ref[s:s + batch])
            o, oc = ora.run(pl[s:s + batch], dm[s:s + batch], ref[s:s + batch])
            stats.append(compare_results(e, o, ec, oc, label=f"[{label}:{s}] "))
        ce, co = eng.counters().as_array(), ora.counters().as_array()
        assert (ce == co).all(), (ce, co)
    eng.close()
    return stats


@pytest.mark.parametrize("numerics", [pm.NUM_PRODUCT, pm.NUM_EXACT, pm.NUM_POLY])
@pytest.mark.parametrize("pedfile,kw", [
    ("test.ped", dict()),
    ("test.ped", dict(min_total_depth=150, max_total_depth=200, posterior=0.9)),
    ("test.mix.ped", dict()),
    ("test.ped", dict(denovo=1, denovo_mut_rate=1.5e-7)),
    ("test.ped", dict(all_sites=1)),
])
def test_example_sites_match_oracle(built, pedfile, kw, numerics):
    ped = pm.Pedigree(os.path.join(EXAMPLE, "test.dat"), os.path.join(EXAMPLE, pedfile))
    secs = _read_all(ped, EXAMPLE)
    stats = _run_both(ped, pm.Params.defaults(numerics=numerics, **kw), secs)
    assert sum(s["sites"] for s in stats) == 81016


def _golden_body(name):
    import gzip
    p = os.path.join(EXAMPLE, name)
    if name.endswith(".gz"):
        return gzip.open(p, "rt").read().splitlines()
    return [l for l in open(p).read().splitlines() if not l.startswith("##")]


@pytest.mark.parametrize("args,golden", [
    (["-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "-c", "0.9", "--minDepth", "150", "--maxDepth", "200",
      "--nthreads", "4"], "test.out.vcf.body.gz"),
    (["-p", "test.mix.ped", "-d", "test.dat", "-g", "test.gif"], "test.out.vcfa.body.gz"),
    (["-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--nthreads", "4", "--denovo", "--rate_denovo", "1.5e-07"],
     "test.denovo.out.vcf"),
])
@pytest.mark.parametrize("numerics", ["product", "exact", "poly"])
def test_cli_reproduces_reference_goldens(built, tmp_path, args, golden, numerics):
    out = tmp_path / "out.vcf"
    r = subprocess.run([pm.BIN_PATH] + args + ["--out_vcf", str(out), "--numerics", numerics], cwd=EXAMPLE,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    got = [l for l in out.read_text().splitlines() if not l.startswith("##")]
    exp = _golden_body(golden)
    assert len(got) == len(exp)
    diff = [i for i, (a, b) in enumerate(zip(got, exp)) if a != b]
    assert not diff, f"{len(diff)} lines differ; first:\n{got[diff[0]][:300]}\n{exp[diff[0]][:300]}"


@pytest.mark.parametrize("shape,nfam,nsites", [("quad", 300, 600), ("trio", 200, 600), ("mixed", 101, 400),
                                               ("single", 64, 300), ("quad", 1500, 160)])
def test_synthetic_device_generator_and_parity(built, shape, nfam, nsites, tmp_path):
    d = str(tmp_path / shape)
    pm.synth_write_dataset(d, shape, nfam, nsites, 7)
    ped = pm.Pedigree(os.path.join(d, "test.dat"), os.path.join(d, "test.ped"))
    secs = _read_all(ped, d)
    label, pos, ref, pl, dm = secs[0]
    # device generator == host generator == GLF files
    hpl, hdm, href = pm.synth_block_host(ped.view, nsites, 7)
    assert (hpl == pl).all() and (hdm == dm).all() and (href == ref).all()
    eng = pm.Engine(ped.view, pm.Params.defaults(), max_batch=nsites)
    d_pl, d_dm, d_ref = eng.alloc(pl.nbytes), eng.alloc(dm.nbytes), eng.alloc(ref.nbytes)
    eng.synth(nsites, 7, 0, d_pl, d_dm, d_ref)
    gpl, gdm, gref = np.zeros_like(pm.planar(pl)), np.zeros_like(dm), np.zeros_like(ref)
    eng.to_host(gpl, d_pl, pl.nbytes); eng.to_host(gdm, d_dm, dm.nbytes); eng.to_host(gref, d_ref, ref.nbytes)
    assert (gpl == pm.planar(pl)).all() and (gdm == dm).all() and (gref == ref).all()   # planar device layout
    # pm_engine_to_planar: person-major device block -> the same planar block
    d_pm, d_pl2 = eng.alloc(pl.nbytes), eng.alloc(pl.nbytes)
    eng.to_device(d_pm, pl, pl.nbytes)
    eng.to_planar(nsites, d_pm, d_pl2)
    gpl2 = np.zeros_like(gpl)
    eng.to_host(gpl2, d_pl2, pl.nbytes)
    assert (gpl2 == gpl).all()
    eng.free(d_pm); eng.free(d_pl2)
    for p in (d_pl, d_dm, d_ref):
        eng.free(p)
    eng.close()
    stats = _run_both(ped, pm.Params.defaults(), secs, batch=256)
    assert sum(s["called"] for s in stats) > 0
    if nfam > 1024:   # 1025-2048 nuclear families: the two-wave 128 x 16 plan
        eng = pm.Engine(ped.view, pm.Params.defaults(), max_batch=16)
        assert eng.plan() == (128, 16)
        eng.close()



@pytest.mark.parametrize("shape,nfam,denovo,nsites", [("quad", 64, 0, 500), ("quad+dn", 64, 1, 500), ("trio+dn", 64, 1, 500),
                                                     ("quad+dn", 300, 1, 300), ("quad+dn", 600, 1, 150), ("trio+dn", 528, 1, 150),
                                                     ("quad+dn", 1200, 1, 96), ("quad+dn", 2100, 1, 64),
                                                     ("trio", 300, 0, 300), ("mixed", 1104, 0, 96), ("quad", 1200, 0, 96),
                                                     ("mixed", 2000, 0, 48)])
def test_plane_prefetch_bit_identical(built, tmp_path, monkeypatch, shape, nfam, denovo, nsites):
    """The lean kernels' LDS staging of the PL bytes (plain: the item's 3 planes, 16-B pieces when n_person % 16 == 0
    and 4-B pieces when only n_person % 4 == 0 -- trio 300: 900 persons, mixed 1104: 3864 -- on one-wave plans and
    on the two-wave 128 x 16 plan of 1025-2048 families; --denovo: per-wave windows of all 10 planes,
    double-buffered by LDS-DMA) gives bit-identical results to the direct-load hoisting (PM_NO_PREFETCH=1) on the
    same lane plan, and both match the oracle."""
    d = str(tmp_path / "pf")
    pm.synth_write_dataset(d, shape, nfam, nsites, 13)   # n_person % 16 == 0
    ped = pm.Pedigree(os.path.join(d, "test.dat"), os.path.join(d, "test.ped"))
    label, pos, ref, pl, dm = _read_all(ped, d)[0]
    params = pm.Params.defaults(numerics=pm.NUM_POLY, denovo=denovo, denovo_mut_rate=1e-5 if denovo else 1.5e-8)
    outs = []
    for nopf in ("", "1"):
        if nopf:
            monkeypatch.setenv("PM_NO_PREFETCH", nopf)
        eng = pm.Engine(ped.view, params, max_batch=len(ref))
        outs.append(eng.run(pl, dm, ref))
        eng.close()
    (a, ac), (b, bc) = outs
    # same lane plan both ways, except for 513-1024 --denovo families (staging selects the 64 x 16 plan there);
    # above 1024 families both take the multi-wave plans (512 x 4, 1024 x 4: 48 / 96 KB of staging buffers)
    if nfam <= 512 or nfam > 1024:
        assert a.tobytes() == b.tobytes() and ac.tobytes() == bc.tobytes()
    o, oc = Oracle(ped.view, params).run(pl, dm, ref)
    assert compare_results(a, o, ac, oc, label="prefetch ")["called"] > 0
    assert compare_results(b, o, bc, oc, label="direct ")["called"] > 0


@pytest.mark.parametrize("nfam,nsites", [(300, 200), (512, 128), (600, 128), (1024, 64)])
def test_quad_plan_matches_oracle(built, tmp_path, monkeypatch, nfam, nsites):
    """QUAD lane plans (every family a 4-person nuclear family in person order, n_person % 16 == 0: the lean de
    novo kernel reads each family's PL bytes as one dword per genotype plane, LDS-DMA ring, prefetch across items,
    factored quartic) against the oracle, and the same sites through the general de novo hoisting (PM_NO_QUAD=1)
    against the oracle too.  300 / 600 families end in a partial slot row (phantom families), 512 / 1024 fill the
    64 x 8 / 64 x 16 plans exactly; planted de novo kids give cfg-7 items as well.  On the QUAD plan the de novo
    monomorphism likelihood (cfg 0) comes from the cfg-1 items' hoisted f^4 coefficients; PM_MONO_DN_PREP=1 forms
    it in k_prep from all ten planes instead: both against the oracle, and within 1e-12 (relative; 1e-13 absolute) of each other."""
    d = str(tmp_path / "qd")
    pm.synth_write_dataset(d, "quad+dn", nfam, nsites, 17)
    ped = pm.Pedigree(os.path.join(d, "test.dat"), os.path.join(d, "test.ped"))
    label, pos, ref, pl, dm = _read_all(ped, d)[0]
    params = pm.Params.defaults(numerics=pm.NUM_POLY, denovo=1, denovo_mut_rate=1e-5)
    o, oc = Oracle(ped.view, params).run(pl, dm, ref)
    got = {}
    for env in ("", "PM_MONO_DN_PREP", "PM_NO_QUAD"):
        if env:
            monkeypatch.setenv(env, "1")
        eng = pm.Engine(ped.view, params, max_batch=len(ref))
        assert eng.plan() == (64, 8 if nfam <= 512 else 16)
        e, ec = eng.run(pl, dm, ref)
        eng.close()
        st = compare_results(e, o, ec, oc, label=(env or "quad") + " ")
        assert st["called"] > 0
        got[env] = e
        if env:
            monkeypatch.delenv(env)
    a, b = got[""], got["PM_MONO_DN_PREP"]
    called = a["status"] == 0   # PM_SITE_CALLED
    np.testing.assert_allclose(a["varllk"][called, 0], b["varllk"][called, 0], rtol=1e-12, atol=1e-13)


@pytest.mark.parametrize("numerics", [pm.NUM_PRODUCT, pm.NUM_POLY])
@pytest.mark.parametrize("shape", ["quad+dn", "trio+dn"])
def test_denovo_planted_parity(built, tmp_path, numerics, shape):
    """--denovo on synthetic nuclear families with planted de novo kids: written records (10-state kid
    posteriors) next to suppressed records (emit 2, no genotype row).  POLY runs the lean polynomial de novo
    kernel, PRODUCT the generic one; both against the oracle."""
    d = str(tmp_path / "dn")
    pm.synth_write_dataset(d, shape, 40, 700, 31)
    ped = pm.Pedigree(os.path.join(d, "test.dat"), os.path.join(d, "test.ped"))
    label, pos, ref, pl, dm = _read_all(ped, d)[0]
    params = pm.Params.defaults(denovo=1, denovo_mut_rate=1e-5, numerics=numerics)
    eng = pm.Engine(ped.view, params, max_batch=len(ref))
    ora = Oracle(ped.view, params)
    e, ec = eng.run(pl, dm, ref)
    o, oc = ora.run(pl, dm, ref)
    st = compare_results(e, o, ec, oc, label="denovo ")
    eng.close()
    assert (o["emit"] == 1).sum() > 0 and (o["emit"] == 2).sum() > 0, np.unique(o["emit"], return_counts=True)
    assert ((e["call_row"] >= 0) == (o["emit"] == 1)).all()
    assert st["called"] > 0


@pytest.mark.parametrize("io_threads", [1, 6])
def test_cli_ragged_glf_matches_reference(built, tmp_path, io_threads):
    """The product CLI (parallel GLF ingest + HIP engine) on ragged GLFs reproduces the reference's VCF."""
    import gzip
    ingest = os.path.join(os.path.dirname(EXAMPLE), "ingest")
    out = tmp_path / "out.vcf"
    r = subprocess.run([pm.BIN_PATH, "-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--all_sites",
                        "--io_threads", str(io_threads), "--out_vcf", str(out)], cwd=ingest, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    got = [l for l in out.read_text().splitlines() if not l.startswith("##")]
    exp = [l for l in gzip.open(os.path.join(ingest, "ref.vcf.body.gz"), "rt").read().splitlines() if l]
    assert got == exp


def test_cli_block_input_reproduces_golden(built, tmp_path):
    """--glf2blocks then --in_blocks through the product CLI (engine on the GPU) gives the reference golden."""
    import gzip
    pmb = str(tmp_path / "example.pmb")
    r = subprocess.run([pm.BIN_PATH, "-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--glf2blocks", pmb], cwd=EXAMPLE,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    out = tmp_path / "out.vcf"
    r = subprocess.run([pm.BIN_PATH, "-p", "test.ped", "-d", "test.dat", "--in_blocks", pmb, "-c", "0.9", "--minDepth", "150",
                        "--maxDepth", "200", "--out_vcf", str(out)], cwd=EXAMPLE, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    got = [l for l in out.read_text().splitlines() if not l.startswith("##")]
    assert got == gzip.open(os.path.join(EXAMPLE, "test.out.vcf.body.gz"), "rt").read().splitlines()


@pytest.mark.parametrize("denovo", [0, 1])
def test_headline_config_parity(built, denovo):
    """The bench's own workload (BASELINE config 3: 1000 nuclear quads, the bench pedigree and site generator,
    the geometry and kernels the bench runs -- one wave per item with 16 family slots per lane: the de novo
    kernel that compiles only the LDS-staged hoisting, or the plain kernel with plane prefetch) against the
    CPU oracle on the first 1024 sites.  The plan is asserted so a geometry change fails loudly here."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    ped = bench.nuclear_pedigree(pm, 1000, 2)
    pl, dm, ref = pm.synth_block_host(ped, 1024, 7)
    params = pm.Params.defaults(denovo=denovo)
    eng = pm.Engine(ped, params, max_batch=1024)
    assert eng.plan() == (64, 16)
    e, ec = eng.run(pl, dm, ref)
    eng.close()
    o, oc = Oracle(ped, params).run(pl, dm, ref)
    st = compare_results(e, o, ec, oc, label="headline ")
    assert st["sites"] == 1024 and st["called"] > 0


@pytest.mark.parametrize("case", ["example", "quad_chrX", "late_chrX", "multi_all"])
def test_cli_two_shards_match_one_process(built, tmp_path, case):
    """polymutt_amd.launch with 2 ranks (here both on the one GPU, gloo for the per-section exchange; RCCL
    when each rank has its own GPU) writes the same VCF and section summaries as the one-process CLI."""
    from test_cpu_host import _sharded_case, run_sharded, summary_lines, vcf_body
    cwd, args = _sharded_case(tmp_path, case)
    one = str(tmp_path / "one.vcf")
    r1 = subprocess.run([pm.BIN_PATH] + args + ["--out_vcf", one], cwd=cwd, capture_output=True, text=True, timeout=300)
    assert r1.returncode == 0, r1.stdout[-2000:]
    sh = str(tmp_path / "sharded.vcf")
    r2 = run_sharded(cwd, args + ["--out_vcf", sh], 2)
    assert r2.returncode == 0, r2.stdout[-3000:] + r2.stderr[-3000:]
    assert vcf_body(sh) == vcf_body(one)
    assert summary_lines(r2.stdout) == summary_lines(r1.stdout) and summary_lines(r1.stdout)
    assert ("first record re-run" in r2.stderr) == (case == "late_chrX")


@pytest.mark.parametrize("case", ["example", "quad_chrX"])
def test_cli_rccl_exchange_world_one(built, tmp_path, monkeypatch, case):
    """The CLI's section exchange (launch.py: the all-gather that replaces src/main.cpp:264-282's summary counters
    and orders the VCF merge) forced onto RCCL at world 1 (PM_COLLECTIVE=nccl): the sharded protocol runs over one
    rank with the all-gather on the GPU, and the VCF and section summaries equal the plain one-process CLI's."""
    from test_cpu_host import _sharded_case, run_sharded, summary_lines, vcf_body
    cwd, args = _sharded_case(tmp_path, case)
    one = str(tmp_path / "one.vcf")
    r1 = subprocess.run([pm.BIN_PATH] + args + ["--out_vcf", one], cwd=cwd, capture_output=True, text=True, timeout=300)
    assert r1.returncode == 0, r1.stdout[-2000:]
    sh = str(tmp_path / "rccl.vcf")
    monkeypatch.setenv("PM_COLLECTIVE", "nccl")
    r2 = run_sharded(cwd, args + ["--out_vcf", sh], 1)
    assert r2.returncode == 0, r2.stdout[-3000:] + r2.stderr[-3000:]
    assert "collective backend nccl, world 1" in r2.stderr, r2.stderr[-2000:]
    assert vcf_body(sh) == vcf_body(one)
    assert summary_lines(r2.stdout) == summary_lines(r1.stdout) and summary_lines(r1.stdout)


def test_posterior_carry_matches_oracle(built, tmp_path):
    """famlk[0]'s stale posterior state (pm_engine_set_posterior_carry) set explicitly, as a shard start does:
    the engine's chrX genotype posteriors follow the oracle's for both states, and the state is visible in
    them (trios: the last person is male, so the stale member sex changes the first family's kid terms)."""
    d = str(tmp_path / "t")
    pm.synth_write_dataset(d, "trio+late", 30, 400, 31)
    ped = pm.Pedigree(os.path.join(d, "test.dat"), os.path.join(d, "test.ped"))
    label, pos, ref, pl, dm = _read_all(ped, d)[0]
    from oracle_binding import lib
    import ctypes as C
    L = lib()
    L.pmo_set_posterior_carry.argtypes = [C.c_void_p, C.c_int32]
    dos = []
    for carry in (0, 1):
        eng = pm.Engine(ped.view, pm.Params.defaults(), max_batch=256)
        ora = Oracle(ped.view, pm.Params.defaults())
        eng.begin_section(pm.PM_CHR_X)
        ora.begin_section(pm.PM_CHR_X)
        eng.set_posterior_carry(carry)
        L.pmo_set_posterior_carry(ora.h, carry)
        e, ec = eng.run(pl[200:456], dm[200:456], ref[200:456])
        o, oc = ora.run(pl[200:456], dm[200:456], ref[200:456])
        compare_results(e, o, ec, oc, label=f"carry={carry} ")
        assert ec.shape[0] > 0
        np.testing.assert_allclose(ec["dosage"], oc["dosage"], rtol=1e-9, atol=1e-300)
        dos.append(ec["dosage"][0].copy())
        eng.close()
    assert (dos[0] != dos[1]).any()   # the first record's posteriors depend on the state


@pytest.mark.parametrize("denovo", [0, 1])
def test_headline_full_batch_properties(built, denovo):
    """BASELINE config 3 at the bench's full batch (1000 quads x 262 144 sites, HBM-resident, k_synth), where
    the oracle cannot follow: size-independent properties.  The same sites in one batch and in four batches
    of 65 536 give bitwise-identical per-site results and section counters (no state leaks between sites or
    batches); every site is called and counted once; the emitted sites are exactly the non-hom-ref calls."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    ped = bench.nuclear_pedigree(pm, 1000, 2)
    B, np_ = 262144, ped.n_person
    params = pm.Params.defaults(denovo=denovo)
    big = pm.Engine(ped, params, max_batch=B)
    d_pl, d_dm, d_ref = big.alloc(B * np_ * 10), big.alloc(B * np_ * 4), big.alloc(B)
    big.synth(B, 7, 0, d_pl, d_dm, d_ref)
    rsz = pm.engine.SITE_DTYPE.itemsize
    d_res = big.alloc(B * rsz)
    big.run_device(B, d_pl, d_dm, d_ref, d_res, None)
    big.sync()
    r_big = np.zeros(B, pm.engine.SITE_DTYPE)
    big.to_host(r_big, d_res, B * rsz)
    c_big = big.counters().as_array()
    small = pm.Engine(ped, params, max_batch=B // 4)
    r_small = np.zeros(B, pm.engine.SITE_DTYPE)
    for k in range(4):   # the same device block, a quarter at a time (planar: site s at s * 10 * n_person)
        off = k * (B // 4)
        sub = lambda p, w: C.c_void_p(p.value + off * w)
        part = np.zeros(B // 4, pm.engine.SITE_DTYPE)
        d_r2 = small.alloc((B // 4) * rsz)
        small.run_device(B // 4, sub(d_pl, np_ * 10), sub(d_dm, np_ * 4), sub(d_ref, 1), d_r2, None)
        small.sync()
        small.to_host(part, d_r2, (B // 4) * rsz)
        small.free(d_r2)
        r_small[off:off + B // 4] = part
    c_small = small.counters().as_array()
    for e, p in ((big, (d_pl, d_dm, d_ref, d_res)), (small, ())):
        for x in p:
            e.free(x)
    big.close()
    small.close()
    keep = [f for f in pm.engine.SITE_DTYPE.names if f != "call_row"]   # row numbers restart per batch
    assert all((r_big[f] == r_small[f]).all() for f in keep)
    assert (c_big == c_small).all()
    assert (r_big["status"] == 0).all() and int(c_big[:5].sum()) == B
    # main.cpp:520-553: every site lands in exactly one filter count or one of homoRef / ts / tv / other / nocall
    assert int(c_big[5:16].sum()) == B
    emitted = r_big["emit"] != 0
    if not denovo:   # records: the polymorphic calls past the posterior cutoff, one per ts / tv / other count
        assert (r_big["maxidx"][emitted] >= 1).all()
        assert int(emitted.sum()) == int(c_big[10:15].sum())


def test_quad_dynamic_item_order_matches_static(built, monkeypatch):
    """The QUAD kernel's dynamic item order (per-XCD claim counters, steals at the end of a list) against the static
    stride order (PM_QD_DYN=0) on a 65 536-site --denovo batch -- lists long enough for claims in every range and
    for steals: bitwise-identical per-site results, section counters and evaluation counts (every item computed
    exactly once, whatever wave took it)."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    ped = bench.nuclear_pedigree(pm, 1000, 2)
    B, np_ = 65536, ped.n_person
    params = pm.Params.defaults(denovo=1)
    out = []
    for dyn in ("0", "1"):
        monkeypatch.setenv("PM_QD_DYN", dyn)
        eng = pm.Engine(ped, params, max_batch=B)
        assert eng.plan() == (64, 16)
        d_pl, d_dm, d_ref = eng.alloc(B * np_ * 10), eng.alloc(B * np_ * 4), eng.alloc(B)
        eng.synth(B, 11, 0, d_pl, d_dm, d_ref)
        rsz = pm.engine.SITE_DTYPE.itemsize
        d_res = eng.alloc(B * rsz)
        eng.kernel_stats(reset=True)
        for _ in range(2):   # (twice: the counters are zeroed per launch)
            eng.run_device(B, d_pl, d_dm, d_ref, d_res, None)
            eng.sync()
        r = np.zeros(B, pm.engine.SITE_DTYPE)
        eng.to_host(r, d_res, B * rsz)
        ks = eng.kernel_stats()
        out.append((r, eng.counters().as_array(), ks.evals, ks.items, ks.launches))
        for x in (d_pl, d_dm, d_ref, d_res):
            eng.free(x)
        eng.close()
    (r0, c0, e0, i0, l0), (r1, c1, e1, i1, l1) = out
    assert all((r0[f] == r1[f]).all() for f in pm.engine.SITE_DTYPE.names), \
        [f for f in pm.engine.SITE_DTYPE.names if not (r0[f] == r1[f]).all()]
    assert (c0 == c1).all() and (e0, i0, l0) == (e1, i1, l1)
    assert int((r1["evals"] > 0).sum()) > 0


def test_bench_rccl_group_of_one(built):
    """bench.py --rccl on the one GPU of the box: the RCCL ("nccl") process group is initialised at one rank and the
    section counters' all-reduce, the barriers and the max-over-ranks timing run through it on the device -- the
    collective path of the multi-GPU bench (src/main.cpp:264-282's summary), exercised without a second GPU."""
    import json
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--rccl", "--steps", "3", "--warmup", "1",
                        "--batch", "8192", "--calib-steps", "1", "--no-cpu-baseline"], capture_output=True, text=True,
                       timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    print("collective_backend:", line["collective_backend"], "rccl_world:", line["rccl_world"])
    assert line["collective_backend"] == "nccl" and line["rccl_world"] == 1
    assert line["counters"]["sites"] == 3 * 8192 and line["value"] > 0


@pytest.mark.parametrize("engines,batch", [(1, 4096), (3, 1000), (2, 257)])
def test_cli_pipelined_engines_reproduce_golden(built, tmp_path, engines, batch):
    """The pipelined CLI with several engines in flight (pm_engine_submit / pm_engine_collect on separate HIP streams,
    page-locked batch buffers, records formatted in parallel and written in order) reproduces the reference's
    example goldens for any engine count and batch size (81 016 sites: 20-316 batches), plain and --denovo."""
    for args, golden in [(["-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "-c", "0.9", "--minDepth", "150",
                           "--maxDepth", "200"], "test.out.vcf.body.gz"),
                         (["-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--denovo", "--rate_denovo", "1.5e-07"],
                          "test.denovo.out.vcf")]:
        out = tmp_path / "out.vcf"
        r = subprocess.run([pm.BIN_PATH] + args + ["--out_vcf", str(out), "--engines", str(engines), "--batch", str(batch)],
                           cwd=EXAMPLE, capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        got = [l for l in out.read_text().splitlines() if not l.startswith("##")]
        assert got == _golden_body(golden), golden


@pytest.mark.parametrize("case", ["quad_chrX", "late_chrX"])
@pytest.mark.parametrize("denovo", [False, True])
def test_cli_engines_chrX_posterior_carry(built, tmp_path, case, denovo):
    """chrX sections over many small batches with several engines: famlk[0]'s stale posterior state passes from one
    engine's batch to the next (EngineEvaluator::note / set_posterior_carry; plain runs take chrX batches one at a
    time), and under --denovo -- where the posterior ignores the carry (d_member_sex_before) and batches stay
    concurrent (in_flight) -- the records equal one engine's, byte for byte."""
    from test_cpu_host import _sharded_case, vcf_body
    cwd, args = _sharded_case(tmp_path, case)
    if denovo:
        args = args + ["--denovo"]
    bodies = []
    for engines in (1, 3):
        out = str(tmp_path / f"e{engines}.vcf")
        r = subprocess.run([pm.BIN_PATH] + args + ["--out_vcf", out, "--engines", str(engines), "--batch", "64"], cwd=cwd,
                           capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        bodies.append(vcf_body(out))
    assert bodies[0] == bodies[1] and len(bodies[0]) > 1


def test_engine_submit_collect_matches_run(built):
    """pm_engine_submit / pm_engine_collect with two engines' batches in flight at once give the same bytes as
    pm_engine_run, batch by batch (the CLI's pipelined engine stage)."""
    import sys
    sys.path.insert(0, ROOT)
    import bench
    ped = bench.nuclear_pedigree(pm, 300, 2)
    pl, dm, ref = pm.synth_block_host(ped, 1024, 5)
    for denovo in (0, 1):
        params = pm.Params.defaults(denovo=denovo)
        engs = [pm.Engine(ped, params, max_batch=512) for _ in range(2)]
        want = [engs[0].run(pl[k * 512:(k + 1) * 512], dm[k * 512:(k + 1) * 512], ref[k * 512:(k + 1) * 512]) for k in range(2)]
        for k in range(2):
            engs[k].begin_section(pm.PM_CHR_AUTO)
            engs[k].submit(pl[k * 512:(k + 1) * 512], dm[k * 512:(k + 1) * 512], ref[k * 512:(k + 1) * 512])
        got = [engs[k].collect() for k in range(2)]
        for (a, ac), (b, bc) in zip(got, want):
            assert a.tobytes() == b.tobytes() and ac.tobytes() == bc.tobytes()
        for e in engs:
            e.close()
