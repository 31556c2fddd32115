"""CPU tests: the oracle (oracle/pm_oracle.c) and the product host driver (GLF reader, pedigree
loader, VCF writer, CLI) pinned against the reference -- its committed example goldens and the
per-site dumps / VCFs of its own objects on synthetic datasets (tests/golden/synth)."""
import gzip
import os
import subprocess

import numpy as np
import pytest

import polymutt_amd as pm
from conftest import EXAMPLE
from fixtures import (CASES, DUMP_CASES, ORACLE_SLOW, compare_to_dump, golden_dump, golden_vcf_body, make_dataset, params_and_chrom,
                      read_dataset, summary_block)
from oracle_binding import Oracle


def _body(path):
    return [l for l in open(path).read().splitlines() if not l.startswith("##")]


EXAMPLE_RUNS = [
    (["-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "-c", "0.9", "--minDepth", "150", "--maxDepth", "200",
      "--nthreads", "4"], "test.out.vcf.body.gz"),
    (["-p", "test.mix.ped", "-d", "test.dat", "-g", "test.gif"], "test.out.vcfa.body.gz"),
    (["-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--nthreads", "4", "--denovo", "--rate_denovo", "1.5e-07"],
     "test.denovo.out.vcf"),
]


@pytest.mark.parametrize("args,golden", EXAMPLE_RUNS, ids=["default_filters", "mix_ped", "denovo"])
def test_cpu_driver_reproduces_example_goldens(cpu_driver, tmp_path, args, golden):
    out = tmp_path / "out.vcf"
    r = subprocess.run([cpu_driver] + args + ["--out_vcf", str(out)], cwd=EXAMPLE, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-2000:]
    p = os.path.join(EXAMPLE, golden)
    exp = gzip.open(p, "rt").read().splitlines() if p.endswith(".gz") else _body(p)
    got = _body(out)
    assert got == exp


@pytest.mark.parametrize("name", [n for n in DUMP_CASES if n not in ORACLE_SLOW])
def test_oracle_matches_reference_dump(built, tmp_path, name):
    case = make_dataset(name, str(tmp_path))
    ped, secs, sha = read_dataset(str(tmp_path))
    assert sha == case["block_sha256"], "synthetic generator no longer reproduces the reference's inputs"
    par, chrom = params_and_chrom(case["flags"])
    ora = Oracle(ped.view, par)
    ora.begin_section(chrom)
    (label, pos, ref, pl, dm), = secs
    res, _ = ora.run(pl, dm, ref)
    st = compare_to_dump(res, golden_dump(name), label=name + " ")
    assert st["sites"] == case["dumped_sites"]
    # same Brent in the same arithmetic order: identical evaluation counts and minimisers
    assert st["eval_path_mismatch"] == 0 and st["flat_divergence"] == 0 and st["nonflat_divergence"] == 0, st


@pytest.mark.parametrize("name", sorted(set(CASES) - ORACLE_SLOW))
def test_cpu_driver_matches_reference_vcf(cpu_driver, tmp_path, name):
    case = make_dataset(name, str(tmp_path))
    r = subprocess.run([cpu_driver, "-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--out_vcf", "out.vcf"]
                       + case["flags"], cwd=tmp_path, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:]
    exp = [l for l in golden_vcf_body(name) if l]
    got = _body(tmp_path / "out.vcf") if os.path.exists(tmp_path / "out.vcf") else []
    assert len(got) == len(exp)
    diff = [i for i, (a, b) in enumerate(zip(got, exp)) if a != b]
    assert not diff, f"{len(diff)} lines differ; first:\n{got[diff[0]][:300]}\n{exp[diff[0]][:300]}"
    if "summary" in case:   # sections, filters and --pos early return (main.cpp:593: no summary) as the reference printed
        assert summary_block(r.stdout) == case["summary"]


def test_cpu_driver_reproduces_vcf_input_golden(cpu_driver, tmp_path):
    """--in_vcf (PedVCF / FamilyLikelihoodSeq_VCF): example/testvcf.in.vcf -> example/testvcf.out.vcf."""
    out = tmp_path / "out.vcf"
    r = subprocess.run([cpu_driver, "-p", "test.ped", "-d", "test.dat", "--in_vcf",
                        os.path.join(EXAMPLE, "testvcf.in.vcf.gz"), "--out_vcf", str(out)], cwd=EXAMPLE,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "Total samples in both VCF and PED files: 12" in r.stdout
    exp = gzip.open(os.path.join(EXAMPLE, "testvcf.out.vcf.body.gz"), "rt").read().splitlines()
    assert _body(out) == exp


INGEST = os.path.join(os.path.dirname(EXAMPLE), "ingest")


@pytest.mark.parametrize("io_threads,serial,env", [(1, False, {}), (4, False, {}), (4, True, {}),
                                                   (4, False, {"PM_GLF_WINDOW": "64"}),
                                                   (6, False, {"PM_GLF_WINDOW": "64", "PM_NO_DECODE_AHEAD": "1"}),
                                                   (3, False, {"PM_GLF_WINDOW": "97", "PM_FILL_CHUNK": "5"})])
def test_cpu_driver_ragged_glf_matches_reference(cpu_driver, tmp_path, io_threads, serial, env):
    """Parallel GLF ingest (host/ingest.cpp), pipelined or serial driver loop, on ragged GLFs -- per-person position sets, offset-0 repeats,
    indel records, an early section end, a person without a GLF key, two sections -- reproduces the VCF the
    reference wrote for the same files (tests/golden/ingest, tools/make_ingest_golden.py), for any thread
    count, merge window (many windows, each merged and decoded ahead of the previous one's fill) and fill chunk."""
    out = tmp_path / "out.vcf"
    r = subprocess.run([cpu_driver, "-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--all_sites",
                        "--io_threads", str(io_threads), "--out_vcf", str(out)], cwd=INGEST, capture_output=True,
                       text=True, timeout=300, env=dict(os.environ, **({"PM_SERIAL": "1"} if serial else {}), **env))
    assert r.returncode == 0, r.stdout[-2000:]
    exp = [l for l in gzip.open(os.path.join(INGEST, "ref.vcf.body.gz"), "rt").read().splitlines() if l]
    assert _body(out) == exp


@pytest.mark.parametrize("block,batch", [("512", "7"), ("4096", "64"), ("100000", "4096")])
def test_cpu_driver_vcf_input_blocks_and_batches(cpu_driver, tmp_path, block, batch):
    """--in_vcf (host/vcf_input.cpp) with small read blocks -- lines longer than the block (the buffer grows), partial
    lines carried over a refill -- and small batches (the flusher's two batch buffers and the writer thread alternate
    many times) reproduces the reference's example/testvcf.out.vcf body byte for byte, from the gzip input and from
    the same text uncompressed (read by pread pieces)."""
    src_gz = os.path.join(EXAMPLE, "testvcf.in.vcf.gz")
    plain = tmp_path / "in.vcf"
    plain.write_bytes(gzip.open(src_gz, "rb").read())
    exp = [l for l in gzip.open(os.path.join(EXAMPLE, "testvcf.out.vcf.body.gz"), "rt").read().splitlines()]
    for src in (src_gz, str(plain)):
        out = tmp_path / "out.vcf"
        r = subprocess.run([cpu_driver, "-p", "test.ped", "-d", "test.dat", "--in_vcf", src, "--out_vcf", str(out), "--batch", batch],
                           cwd=EXAMPLE, capture_output=True, text=True, timeout=300, env=dict(os.environ, PM_VCF_BLOCK=block))
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        got = [l for l in out.read_text().splitlines() if not l.startswith("##")]
        assert got == exp, src


def test_vcf_fixed_point_formatting_matches_printf(tmp_path):
    """host/vcf_fmt.h (the allocation-free DS/GQ/DP/PL column formatter) prints exactly what glibc's printf
    prints: random dosages, exact decimal ties and their neighbours, signed zeros, subnormals."""
    exe = str(tmp_path / "fmt_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", exe, os.path.join(os.path.dirname(__file__), "native", "fmt_check.cpp")],
                   check=True)
    r = subprocess.run([exe, "300000"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout[-2000:]


@pytest.mark.parametrize("args,golden", EXAMPLE_RUNS[:1] + EXAMPLE_RUNS[2:], ids=["default_filters", "denovo"])
def test_cpu_driver_block_format_round_trip(cpu_driver, tmp_path, args, golden):
    """GLF -> dense indexed blocks (--glf2blocks) -> analysis (--in_blocks) reproduces the reference golden;
    the block index (polymutt_amd/blocks.py) addresses every block and matches the GLF site stream."""
    from polymutt_amd import blocks
    pmb = str(tmp_path / "example.pmb")
    r = subprocess.run([cpu_driver, "-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--glf2blocks", pmb,
                        "--block_sites", "5000"], cwd=EXAMPLE, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:]
    idx = blocks.read_index(pmb)
    secs = blocks.read_sections(pmb)
    assert sum(e["n"] for e in idx) == 81016 and len(secs) >= 1
    ped = pm.Pedigree(os.path.join(EXAMPLE, "test.dat"), os.path.join(EXAMPLE, "test.ped"))
    cwd = os.getcwd()
    os.chdir(EXAMPLE)
    try:
        rd = pm.GlfReader(ped, "test.gif")
        parts = [rd.read(200000) for _ in rd.sections()]
    finally:
        os.chdir(cwd)
    pos, ref, pl, dm = (np.concatenate([p[k].reshape(len(p[1]), -1) if k >= 2 else p[k] for p in parts]) for k in range(4))
    got = [blocks.read_block(pmb, e) for e in idx]
    assert np.array_equal(np.concatenate([g[0] for g in got]) + 1, pos)
    assert np.array_equal(np.concatenate([g[1] for g in got]), ref)
    assert np.array_equal(np.concatenate([g[2] for g in got]), pl.reshape(len(ref), -1, 10))
    assert np.array_equal(np.concatenate([g[3] for g in got]), dm.reshape(len(ref), -1))
    out = tmp_path / "out.vcf"
    blk_args = [a for a in args]
    i = blk_args.index("-g")
    blk_args[i:i + 2] = ["--in_blocks", pmb]
    r = subprocess.run([cpu_driver] + blk_args + ["--out_vcf", str(out)], cwd=EXAMPLE, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout[-2000:]
    p = os.path.join(EXAMPLE, golden)
    exp = gzip.open(p, "rt").read().splitlines() if p.endswith(".gz") else _body(p)
    assert _body(out) == exp


def test_block_file_rejects_mismatched_or_truncated_input(cpu_driver, tmp_path):
    """--in_blocks fails loudly (reference-style FATAL ERROR, exit 1) on a block file written for another
    pedigree size or cut short, instead of analysing garbage."""
    pmb = str(tmp_path / "ragged.pmb")
    r = subprocess.run([cpu_driver, "-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--glf2blocks", pmb],
                       cwd=INGEST, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:]
    raw = open(pmb, "rb").read()
    cut = str(tmp_path / "cut.pmb")
    open(cut, "wb").write(raw[: len(raw) // 2])
    r = subprocess.run([cpu_driver, "-p", "test.ped", "-d", "test.dat", "--in_blocks", cut, "--out_vcf", str(tmp_path / "o.vcf")],
                       cwd=INGEST, capture_output=True, text=True, timeout=300)
    assert r.returncode == 1 and "FATAL ERROR" in r.stdout and "truncated" in r.stdout
    r = subprocess.run([cpu_driver, "-p", os.path.join(EXAMPLE, "test.ped"), "-d", os.path.join(EXAMPLE, "test.dat"),
                        "--in_blocks", pmb, "--out_vcf", str(tmp_path / "o2.vcf")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 1 and "persons" in r.stdout


def test_cpu_driver_vcf_input_record_kinds(cpu_driver, tmp_path):
    """--in_vcf with multi-allelic, REF == ALT, indel and lower-case records (tests/vcf_edits.py) through the
    product host driver on the CPU oracle: drop rules, indel alleles and QUAL pinned against the golden."""
    from vcf_edits import check_edited_output, write_edited_vcf
    src = str(tmp_path / "in.vcf")
    write_edited_vcf(src)
    out = tmp_path / "out.vcf"
    r = subprocess.run([cpu_driver, "-p", "test.ped", "-d", "test.dat", "--in_vcf", src, "--out_vcf", str(out)],
                       cwd=EXAMPLE, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    check_edited_output([l for l in out.read_text().splitlines() if not l.startswith("#")])
