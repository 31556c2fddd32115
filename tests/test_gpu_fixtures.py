"""GPU parity against the reference itself: for every reference-pinned synthetic case
(tests/golden/synth, from the reference's own objects) the HIP engine's per-site results match the
reference's --dump_sites records, its genotype calls match the oracle's, and the product CLI writes
the reference's VCF byte-for-byte."""
import os
import subprocess

import pytest

import polymutt_amd as pm
from fixtures import (CASES, DUMP_CASES, ORACLE_SLOW, compare_to_dump, golden_dump, golden_vcf_body, make_dataset, params_and_chrom,
                      read_dataset, summary_block)
from oracle_binding import Oracle
from parity import compare_results

pytestmark = pytest.mark.gpu


# "big_*" cases are BASELINE.json config geometries (1000 trios, 1000 quads --denovo, 200 ext10 pedigrees,
# extended pedigrees next to > 512 nuclear families): the lane plans and kernel instantiations the bench
# selects for those shapes.  They run in the default numerics only (the oracle needs ~45 s for 200 ext10
# --denovo) and in one batch per 128 sites like the rest.
_DUMP_CASES = [(n, num) for n in DUMP_CASES for num in
               ([pm.NUM_POLY] if n.startswith("big_") else [pm.NUM_PRODUCT, pm.NUM_EXACT, pm.NUM_POLY])]


@pytest.mark.parametrize("name,numerics", _DUMP_CASES)
def test_engine_matches_reference_dump(built, tmp_path, name, numerics):
    case = make_dataset(name, str(tmp_path))
    ped, secs, sha = read_dataset(str(tmp_path))
    assert sha == case["block_sha256"]
    par, chrom = params_and_chrom(case["flags"], numerics=numerics)
    (label, pos, ref, pl, dm), = secs
    eng = pm.Engine(ped.view, par, max_batch=128)
    ora = None if name in ORACLE_SLOW else Oracle(ped.view, par)   # (ORACLE_SLOW: the reference dump alone)
    eng.begin_section(chrom)
    if ora:
        ora.begin_section(chrom)
    res, calls = [], []
    for s in range(0, len(ref), 128):   # several batches: results must not depend on batching
        e, ec = eng.run(pl[s:s + 128], dm[s:s + 128], ref[s:s + 128])
        if ora:
            o, oc = ora.run(pl[s:s + 128], dm[s:s + 128], ref[s:s + 128])
            compare_results(e, o, ec, oc, label=f"{name}[{s}] ")
        res.append(e)
    import numpy as np
    res = np.concatenate(res)
    compare_to_dump(res, golden_dump(name), label=name + " ")
    if ora:
        assert (eng.counters().as_array() == ora.counters().as_array()).all()
    eng.close()


@pytest.mark.parametrize("name", sorted(CASES))
@pytest.mark.parametrize("numerics", ["product", "poly"])
def test_cli_matches_reference_vcf(built, tmp_path, name, numerics):
    case = make_dataset(name, str(tmp_path))
    r = subprocess.run([pm.BIN_PATH, "-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--out_vcf", "out.vcf",
                        "--numerics", numerics] + case["flags"], cwd=tmp_path, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:]
    exp = [l for l in golden_vcf_body(name) if l]
    p = tmp_path / "out.vcf"
    got = [l for l in p.read_text().splitlines() if not l.startswith("##")] if p.exists() else []
    assert len(got) == len(exp)
    diff = [i for i, (a, b) in enumerate(zip(got, exp)) if a != b]
    assert not diff, f"{len(diff)} lines differ; first:\n{got[diff[0]][:300]}\n{exp[diff[0]][:300]}"
    if "summary" in case:   # sections, filters and --pos early return (main.cpp:593: no summary) as the reference printed
        assert summary_block(r.stdout) == case["summary"]


_ES_CASES = [n for n in DUMP_CASES if n.startswith(("ext10", "roof", "roof2", "extmix", "big_ext10", "big_extmix", "big_quadext"))
             and "denovo" not in n]


@pytest.mark.parametrize("name", _ES_CASES)
def test_es_hoisting_kernels_agree(built, tmp_path, monkeypatch, name):
    """The three paths of the polynomial-form Elston-Stewart peel -- the fused compiled kernel (ep_brent_jit: hoisting
    into registers + Brent in one launch, the default for bi-allelic engines whose every family is peeled), the
    compiled hoisting kernel es_hoist_jit + k_brent (PM_NO_FUSED=1) and the generic wave-per-family kernel k_es_hoist
    (PM_NO_JIT=1) -- all match the reference dump of every extended-pedigree case (all chromosome classes the fixtures
    hold)."""
    import numpy as np
    case = make_dataset(name, str(tmp_path))
    ped, secs, _ = read_dataset(str(tmp_path))
    par, chrom = params_and_chrom(case["flags"], numerics=pm.NUM_POLY)
    (label, pos, ref, pl, dm), = secs
    out, rows = {}, {}
    for mode in ("fused", "jit", "generic"):
        if mode == "jit":
            monkeypatch.setenv("PM_NO_FUSED", "1")
        if mode == "generic":
            monkeypatch.setenv("PM_NO_JIT", "1")
        eng = pm.Engine(ped.view, par, max_batch=256)
        eng.begin_section(chrom)
        runs = [eng.run(pl[s:s + 256], dm[s:s + 256], ref[s:s + 256]) for s in range(0, len(ref), 256)]
        eng.close()
        out[mode] = np.concatenate([r[0] for r in runs])
        rows[mode] = [r[1] for r in runs]
        compare_to_dump(out[mode], golden_dump(name), label=f"{name} {mode} ")
    for k in ("status", "n_cfg", "maxidx", "emit"):
        assert (out["jit"][k] == out["generic"][k]).all() and (out["fused"][k] == out["jit"][k]).all(), k
    # genotype rows: the compiled posterior peels follow the reference-order peel term by term -- bit-identical
    # (unless a flat-objective minimiser divergence moved the posterior frequency: af compared to the dump above)
    if (out["jit"]["af"] == out["generic"]["af"]).all():
        for a, b in zip(rows["jit"], rows["generic"]):
            assert a.shape == b.shape and (a == b).all()


_SP3_CASES = [n for n in DUMP_CASES if n.startswith(("roof", "roof2", "extmix", "big_extmix")) and "denovo" in n]


@pytest.mark.parametrize("switch", ["PM_ES_SP3", "PM_ES_T3Z"])
@pytest.mark.parametrize("name", _SP3_CASES)
def test_es_type3_founder_sparsity_is_bit_exact(built, tmp_path, monkeypatch, name, switch):
    """--denovo 10-state peels: the schedule compiler's sparse type-3 sums give the same results bit for bit as the
    dense ones, and both match the reference dump.  PM_ES_SP3: founder-sparse steps (a roof parent that is a founder has
    only its prior's 1-3 states; the pairs outside them add +0) against all 100 pairs; PM_ES_T3Z: the non-founder
    steps' child sums over the Mendelian table's non-zero parent pairs only (the rest add +0) against the 100-pair
    loop."""
    import numpy as np
    case = make_dataset(name, str(tmp_path))
    ped, secs, _ = read_dataset(str(tmp_path))
    par, chrom = params_and_chrom(case["flags"], numerics=pm.NUM_POLY)
    (label, pos, ref, pl, dm), = secs
    out = {}
    for mode in ("sparse", "dense"):
        if mode == "dense":
            monkeypatch.setenv(switch, "0")
        eng = pm.Engine(ped.view, par, max_batch=256)
        eng.begin_section(chrom)
        runs = [eng.run(pl[s:s + 256], dm[s:s + 256], ref[s:s + 256]) for s in range(0, len(ref), 256)]
        eng.close()
        out[mode] = (np.concatenate([r[0] for r in runs]), [r[1] for r in runs])
        compare_to_dump(out[mode][0], golden_dump(name), label=f"{name} {mode} ")
    a, b = out["sparse"][0], out["dense"][0]
    assert a.tobytes() == b.tobytes()
    for x, y in zip(out["sparse"][1], out["dense"][1]):
        assert x.tobytes() == y.tobytes()
