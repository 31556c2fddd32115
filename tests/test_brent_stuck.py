"""Brent failure at site granularity: ScalarMinimizer::Brent's ITMAX exit (core/MathGold.cpp:98,175 -> numerror, which
prints "FATAL NUMERIC ERROR - ScalarMinimizer::Brent got stuck" and exits) ends the reference's run at the stuck site,
with every earlier record already written (fflush per record, src/NucFamGenotypeLikelihood.cpp:1829; PedVCF.cpp prints
record by record) and no summary for the section.  PM_TEST_ITMAX lowers ITMAX (200) in the engine and in the oracle
alike, so the path can be forced: a Brent item needing m loop evaluations gets stuck iff m >= ITMAX, and m = evals - 3
(f(a), f(b), f(c) are counted before the loop), which a normal run reports per site and configuration."""
import os
import subprocess

import numpy as np
import pytest

import polymutt_amd as pm
from conftest import EXAMPLE
from fixtures import make_dataset, read_dataset, params_and_chrom
from oracle_binding import Oracle

FATAL = "FATAL NUMERIC ERROR - ScalarMinimizer::Brent got stuck"


def first_stuck(res, itmax):
    """The first site with a Brent item of >= itmax loop evaluations (-1: none)."""
    ev = res["evals"]
    stuck = ((ev >= 3) & (ev - 3 >= itmax)).any(axis=1)
    idx = np.nonzero(stuck)[0]
    return int(idx[0]) if len(idx) else -1


def pick_itmax(res):
    """An ITMAX whose first stuck site lies nearest the middle of the run (so records exist on both sides)."""
    ev = res["evals"]
    m = np.where(ev >= 3, ev - 3, -1).max(axis=1)
    best = None
    for k in sorted(set(int(x) for x in m if x > 0)):
        s = first_stuck(res, k)
        if s > 0 and (best is None or abs(s - len(res) / 2) < abs(best[1] - len(res) / 2)):
            best = (k, s)
    assert best is not None
    return best


def _body(path):
    return [l for l in open(path).read().splitlines() if not l.startswith("##")] if os.path.exists(path) else []


def _records_before(body, pos):
    """The header line and the records at positions below pos (one section "1")."""
    return body[:1] + [l for l in body[1:] if int(l.split("\t")[1]) < pos]


def _cpu_dataset(tmp_path):
    d = str(tmp_path / "data")
    case = make_dataset("quad_auto", d)
    ped, secs, _ = read_dataset(d)
    (label, pos, ref, pl, dm), = secs
    par, chrom = params_and_chrom(case["flags"])
    ora = Oracle(ped.view, par)
    ora.begin_section(chrom)
    res, _ = ora.run(pl, dm, ref)
    return d, pos, res


def test_cpu_driver_writes_records_before_the_stuck_site(cpu_driver, tmp_path, monkeypatch):
    """The product driver (serial and pipelined) over the CPU oracle: the records of every site before the stuck one
    -- in earlier batches and in the stuck site's own batch -- then the FATAL text, exit status 1, no summary."""
    d, pos, res = _cpu_dataset(tmp_path)
    k, s = pick_itmax(res)
    args = [cpu_driver, "-p", "test.ped", "-d", "test.dat", "-g", "test.gif"]
    r0 = subprocess.run(args + ["--out_vcf", "full.vcf"], cwd=d, capture_output=True, text=True, timeout=600)
    assert r0.returncode == 0, r0.stdout[-2000:]
    full = _body(os.path.join(d, "full.vcf"))
    want = _records_before(full, int(pos[s]))
    assert 1 < len(want) < len(full), (k, s, len(want), len(full))
    for batch, serial in [(64, False), (64, True), (400, False), (7, False)]:
        env = dict(os.environ, PM_TEST_ITMAX=str(k))
        if serial:
            env["PM_SERIAL"] = "1"
        out = f"stuck_{batch}_{int(serial)}.vcf"
        r = subprocess.run(args + ["--out_vcf", out, "--batch", str(batch)], cwd=d, capture_output=True, text=True,
                           timeout=600, env=env)
        assert r.returncode == 1, r.stdout[-2000:]
        assert FATAL in r.stdout and "Summary of reference" not in r.stdout, r.stdout[-2000:]
        assert _body(os.path.join(d, out)) == want, (batch, serial)


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_driver_stops_at_the_stuck_site_gloo(cpu_driver, tmp_path, world):
    """Site shards over gloo: the shard holding the stuck site writes its records before it, the exchange tells every
    rank, the merge keeps the earlier shards and drops the later ones: the one-process output, exit status 1."""
    from test_cpu_host import run_sharded
    d, pos, res = _cpu_dataset(tmp_path)
    k, s = pick_itmax(res)
    args = ["-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--batch", "64"]
    env = dict(os.environ, PM_TEST_ITMAX=str(k))
    r1 = subprocess.run([cpu_driver] + args + ["--out_vcf", "one.vcf"], cwd=d, capture_output=True, text=True, timeout=600,
                        env=env)
    assert r1.returncode == 1 and FATAL in r1.stdout
    os.environ["PM_TEST_ITMAX"] = str(k)
    try:
        lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "native", "build",
                           "libpm_cpu_driver.so")
        r2 = run_sharded(d, args + ["--out_vcf", "sharded.vcf"], world, lib=lib)
    finally:
        del os.environ["PM_TEST_ITMAX"]
    assert r2.returncode != 0
    assert FATAL in r2.stdout, r2.stdout[-2000:] + r2.stderr[-2000:]
    assert _body(os.path.join(d, "sharded.vcf")) == _body(os.path.join(d, "one.vcf"))
    assert not [f for f in os.listdir(d) if ".part" in f]


@pytest.mark.parametrize("world", [1, 2])
def test_vcf_input_stops_at_the_stuck_record(cpu_driver, tmp_path, world):
    """--in_vcf: the records before the stuck one (computed or printed with a carried state) are written, whatever the
    batch size or shard count; the output is a strict prefix of the normal run's."""
    args = ["-p", "test.ped", "-d", "test.dat", "--in_vcf", os.path.join(EXAMPLE, "testvcf.in.vcf.gz")]
    full = str(tmp_path / "full.vcf")
    r0 = subprocess.run([cpu_driver] + args + ["--out_vcf", full], cwd=EXAMPLE, capture_output=True, text=True, timeout=600)
    assert r0.returncode == 0
    fb = _body(full)
    outs = []
    for batch in (5, 256, 4096):
        out = str(tmp_path / f"stuck{batch}.vcf")
        env = dict(os.environ, PM_TEST_ITMAX="12")
        if world == 1:
            r = subprocess.run([cpu_driver] + args + ["--out_vcf", out, "--batch", str(batch)], cwd=EXAMPLE,
                               capture_output=True, text=True, timeout=600, env=env)
        else:
            from test_cpu_host import run_sharded
            os.environ["PM_TEST_ITMAX"] = "12"
            try:
                lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "native", "build",
                                   "libpm_cpu_driver.so")
                r = run_sharded(EXAMPLE, args + ["--out_vcf", out, "--batch", str(batch)], world, lib=lib)
            finally:
                del os.environ["PM_TEST_ITMAX"]
        assert r.returncode != 0 and FATAL in r.stdout, r.stdout[-2000:]
        outs.append(_body(out))
    assert outs[0] == outs[1] == outs[2]
    assert 1 < len(outs[0]) < len(fb) and fb[:len(outs[0])] == outs[0]


@pytest.mark.gpu
def test_engine_reports_the_first_stuck_site(built, tmp_path, monkeypatch):
    """pm_engine_run under PM_TEST_ITMAX: PM_EBRENT with pm_engine_stuck_site = the first site whose Brent needs that
    many loop evaluations (from the normal run's counts), the results and genotype rows before it unchanged."""
    d = str(tmp_path / "data")
    case = make_dataset("quad_auto", d)
    ped, secs, _ = read_dataset(d)
    (label, pos, ref, pl, dm), = secs
    par, chrom = params_and_chrom(case["flags"])
    eng = pm.Engine(ped.view, par, max_batch=len(ref))
    eng.begin_section(chrom)
    res, calls = eng.run(pl, dm, ref)
    assert eng.stuck_site() == -1
    eng.close()
    k, s = pick_itmax(res)
    monkeypatch.setenv("PM_TEST_ITMAX", str(k))
    eng = pm.Engine(ped.view, par, max_batch=len(ref))
    eng.begin_section(chrom)
    with pytest.raises(pm.engine.BrentStuck) as ei:
        eng.run(pl, dm, ref)
    e = ei.value
    assert e.site == s == eng.stuck_site()
    for f in ("status", "emit", "maxidx", "n_cfg", "call_row", "evals"):
        assert (e.results[f][:s] == res[f][:s]).all(), f
    assert (e.results["varllk"][:s] == res["varllk"][:s]).all()
    nrows = int((res["call_row"][:s] >= 0).sum())
    assert len(e.calls) == nrows and (e.calls == calls[:nrows]).all()
    eng.close()


@pytest.mark.gpu
def test_cli_writes_records_before_the_stuck_site(built, tmp_path):
    """The GPU CLI (pipelined, several engines) under PM_TEST_ITMAX: the normal run's VCF truncated just before the
    stuck site's record, then the reference's FATAL text and exit status 1."""
    d = str(tmp_path / "data")
    case = make_dataset("quad_auto", d)
    ped, secs, _ = read_dataset(d)
    (label, pos, ref, pl, dm), = secs
    par, chrom = params_and_chrom(case["flags"])
    eng = pm.Engine(ped.view, par, max_batch=len(ref))
    eng.begin_section(chrom)
    res, _ = eng.run(pl, dm, ref)
    eng.close()
    k, s = pick_itmax(res)
    args = [pm.BIN_PATH, "-p", "test.ped", "-d", "test.dat", "-g", "test.gif"]
    r0 = subprocess.run(args + ["--out_vcf", "full.vcf"], cwd=d, capture_output=True, text=True, timeout=600)
    assert r0.returncode == 0, r0.stdout[-2000:]
    full = _body(os.path.join(d, "full.vcf"))
    want = _records_before(full, int(pos[s]))
    assert 1 < len(want) < len(full)
    for batch in (64, 400):
        out = f"stuck{batch}.vcf"
        r = subprocess.run(args + ["--out_vcf", out, "--batch", str(batch)], cwd=d, capture_output=True, text=True,
                           timeout=600, env=dict(os.environ, PM_TEST_ITMAX=str(k)))
        assert r.returncode == 1, r.stdout[-2000:]
        assert FATAL in r.stdout and "Summary of reference" not in r.stdout
        assert _body(os.path.join(d, out)) == want, batch
