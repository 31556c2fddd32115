"""CPU tests of the drop-in boundary and the host side: the C-ABI library loads and exports every
entry point include/*.h declares, the product fails loudly without a HIP device, the pedigree loader
and Elston-Stewart schedule builder reproduce the reference's ordering, the
synthetic generator is identical between its host and GLF-file forms, and site sharding plus the
single counter all-reduce equals the unsharded section (gloo, world_size 2)."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import polymutt_amd as pm
from conftest import EXAMPLE, ROOT
from polymutt_amd.shard import shard_range

HEADERS = [os.path.join(ROOT, "include", h) for h in ("polymutt_engine.h", "polymutt_host.h")]


def _declared_functions():
    names = set()
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(pmh?_\w+)\s*\(", text, flags=re.M):
            names.add(m.group(1))
    return names


def _gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def test_library_exports_every_declared_entry_point():
    declared = _declared_functions()
    assert len(declared) >= 25, declared
    lib = C.CDLL(pm.LIB_PATH)
    missing = [n for n in sorted(declared) if not hasattr(lib, n)]
    assert not missing, missing
    # the Python binding declares exactly the header's surface
    assert declared == set(pm.engine.EXPORTS), declared ^ set(pm.engine.EXPORTS)
    nm = subprocess.run(["nm", "-D", "--defined-only", pm.LIB_PATH], capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in nm.splitlines() if " T " in l}
    assert declared <= exported


def test_abi_version_and_struct_layout():
    lib = pm.load_library()
    src = open(HEADERS[0]).read()
    ver = int(re.search(r"#define PM_ABI_VERSION (\d+)", src).group(1))
    assert lib.pm_abi_version() == ver
    assert C.sizeof(pm.SiteResult) == 240 and C.sizeof(pm.GenoCall) == 16
    assert C.sizeof(pm.Counters) == 16 * 8


@pytest.mark.skipif(_gpu(), reason="checks the no-device failure path")
def test_engine_fails_loudly_without_device():
    ped = pm.Pedigree(os.path.join(EXAMPLE, "test.dat"), os.path.join(EXAMPLE, "test.ped"))
    with pytest.raises(RuntimeError, match="no HIP device"):
        pm.Engine(ped.view, pm.Params.defaults())


@pytest.mark.skipif(_gpu(), reason="checks the no-device failure path")
def test_cli_fails_loudly_without_device(tmp_path):
    r = subprocess.run([pm.BIN_PATH, "-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--out_vcf",
                        str(tmp_path / "o.vcf")], cwd=EXAMPLE, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "FATAL ERROR" in r.stdout and "HIP device" in r.stdout
    assert not (tmp_path / "o.vcf").exists() or "#CHROM" not in (tmp_path / "o.vcf").read_text()


def test_cli_rejects_unknown_option():
    r = subprocess.run([pm.BIN_PATH, "--no_such_flag"], capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "FATAL ERROR" in r.stdout


def test_example_pedigree_layout():
    ped = pm.Pedigree(os.path.join(EXAMPLE, "test.dat"), os.path.join(EXAMPLE, "test.ped"))
    assert ped.n_fam == 3 and ped.n_person == 12
    assert list(ped.fam_start()) == [0, 4, 8, 12]
    assert list(ped.fam_kind()) == [pm.FAM_NUCLEAR] * 3
    assert list(ped.sex()[:4]) == [1, 2, 1, 2] or set(ped.sex()) <= {1, 2}
    mix = pm.Pedigree(os.path.join(EXAMPLE, "test.dat"), os.path.join(EXAMPLE, "test.mix.ped"))
    kinds = list(mix.fam_kind())
    assert kinds.count(pm.FAM_NUCLEAR) == 2 and kinds.count(pm.FAM_FOUNDERS) == 4


def _steps(ped, f):
    v = ped.view
    ps = np.ctypeslib.as_array(v.peel_start, shape=(v.n_fam + 1,))
    return [(v.steps[i].type, v.steps[i].from0, v.steps[i].from1, v.steps[i].to0, v.steps[i].to1)
            for i in range(ps[f], ps[f + 1])]


@pytest.mark.parametrize("shape,expected", [
    # SURVEY.md Appendix C, observed with the reference's own ES_Peeling
    ("ext10", [(1, 6, -1, 4, 2), (1, 7, -1, 4, 2), (1, 8, -1, 3, 5), (1, 9, -1, 3, 5), (2, 2, -1, 4, -1),
               (2, 3, -1, 5, -1), (1, 4, -1, 0, 1), (1, 5, -1, 0, 1), (2, 0, -1, 1, -1)]),
    ("roof", [(1, 6, -1, 4, 5), (1, 7, -1, 4, 5), (3, 0, 1, 4, -1), (3, 2, 3, 5, -1), (2, 4, -1, 5, -1)]),
    # traced by hand through ES_Peeling::BuildPeelingOrder (FamilyLikelihoodES.cpp:135-277): the roof (7, 6) is
    # created by UpdateRoof after the type-3 peel into 7 and keyed like the marriage partial of leaf 8
    ("roof2", [(1, 8, -1, 7, 6), (1, 11, -1, 9, 10), (3, 0, 1, 6, -1), (3, 2, 3, 7, -1), (3, 4, 5, 10, -1),
               (3, 7, 6, 9, -1), (2, 10, -1, 9, -1)]),
])
def test_peeling_schedule_matches_reference(tmp_path, shape, expected):
    pm.synth_write_dataset(str(tmp_path), shape, 2, 1, 1)
    ped = pm.Pedigree(str(tmp_path / "test.dat"), str(tmp_path / "test.ped"))
    assert list(ped.fam_kind()) == [pm.FAM_EXTENDED] * 2
    for f in range(2):
        assert _steps(ped, f) == expected


def test_synthetic_host_block_equals_glf_files(tmp_path):
    from fixtures import read_dataset
    for shape, nfam in [("quad", 13), ("mixed", 9), ("ext10", 3), ("single", 5)]:
        d = tmp_path / shape
        pm.synth_write_dataset(str(d), shape, nfam, 97, 5)
        ped, secs, _ = read_dataset(str(d))
        (label, pos, ref, pl, dm), = secs
        assert label == "1" and (np.diff(pos) == 1).all()
        hpl, hdm, href = pm.synth_block_host(ped.view, 97, 5)
        assert (hpl == pl).all() and (hdm == dm).all() and (href == ref).all()
        # depth U{8..29}, mapQ 60, PL 255 outside the 3 biallelic genotypes
        depth, mq = dm & 0xFFFFFF, dm >> 24
        assert depth.min() >= 8 and depth.max() <= 29 and (mq == 60).all()
        assert ((pl == 255).sum(axis=-1) >= 7).all() and (pl.min(axis=-1) == 0).all()


def test_shard_range_partitions():
    for n in (0, 1, 7, 1000, 1001):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= 1


@pytest.mark.parametrize("gpus", [1, 2, 3])
def test_bench_gpus_flag_launches_that_many_ranks(gpus):
    """`bench.py --gpus N` run directly (no WORLD_SIZE) starts N worker processes itself and the collective
    sees all of them (dry run: gloo, no engine)."""
    import json
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=dict(env, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == gpus and line["rccl_world"] == gpus
    assert line["counter_sum"] == gpus * (gpus + 1) // 2   # every rank's counters reached the all-reduce


def test_bench_rejects_world_mismatch():
    import sys
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_sharded(cwd, args, world, lib=None, timeout=600):
    """polymutt_amd.launch under torchrun: `world` one-process shards of the product driver (lib: another
    pmh_run_polymutt build, e.g. the CPU-oracle one).  Returns the CompletedProcess."""
    import sys
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(world),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m", "polymutt_amd.launch"]
    cmd += (["--lib", lib] if lib else []) + list(args)
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""), OMP_NUM_THREADS="1")
    return subprocess.run(cmd, cwd=cwd, capture_output=True, text=True, timeout=timeout, env=env)


def summary_lines(stdout):
    """The section summaries a run prints (main.cpp:596-619), without the wall-clock lines."""
    keep, on = [], False
    for l in stdout.splitlines():
        if l.startswith("Summary of reference"):
            on = True
        if on and l.strip() and not l.startswith(("Analysis ended", "Running time")):
            keep.append(l)
    return keep


def vcf_body(path):
    return [l for l in open(path).read().splitlines() if not l.startswith("##")]


def _sharded_case(tmp_path, case):
    from conftest import EXAMPLE
    import shutil
    if case == "example":
        return EXAMPLE, ["-p", "test.ped", "-d", "test.dat", "-g", "test.gif"]
    if case == "ragged":
        return os.path.join(os.path.dirname(EXAMPLE), "ingest"), ["-p", "test.ped", "-d", "test.dat", "-g", "test.gif",
                                                                  "--all_sites"]
    d = str(tmp_path / case)
    if case == "quad_chrX":
        from fixtures import make_dataset
        make_dataset("quad_chrX", d)
        return d, ["-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--chrX", "1"]
    if case in ("multi_all", "multi_chr2process"):   # three sections (1, X, 2): the exchange once per section
        from fixtures import make_dataset
        c = make_dataset(case, d)
        return d, ["-p", "test.ped", "-d", "test.dat", "-g", "test.gif"] + c["flags"]
    if case == "late_chrX":   # shard 0 emits nothing: shard 1 must redo its first record with famlk[0] unseen
        pm.synth_write_dataset(d, "trio+late", 30, 400, 31)   # (trios: the last person is male, so the state matters)
        return d, ["-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--chrX", "1"]
    raise ValueError(case)


@pytest.mark.parametrize("case,world,block_sites", [("example", 2, 5000), ("example", 2, 10127), ("example", 3, 7000), ("multi_all", 2, 64),
                                                    ("multi_chr2process", 3, 50), ("late_chrX", 2, 37)])
def test_sharded_blocks_seek_to_their_range(cpu_driver, tmp_path, case, world, block_sites):
    """Block input (--in_blocks) under the multi-process driver: each rank seeks by the block index to the first
    block of its position range and skips the rest of a section after it, so it reads exactly the blocks that
    overlap its range (none wholly below lo, none wholly at or past hi), and the merged VCF and summaries equal
    one process's."""
    from polymutt_amd import blocks
    cwd, args = _sharded_case(tmp_path, case)
    pmb = str(tmp_path / "in.pmb")
    r = subprocess.run([cpu_driver] + args + ["--glf2blocks", pmb, "--block_sites", str(block_sites)], cwd=cwd,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:]
    i = args.index("-g")
    bargs = args[:i] + ["--in_blocks", pmb] + args[i + 2:]
    one = str(tmp_path / "one.vcf")
    r1 = subprocess.run([cpu_driver] + bargs + ["--out_vcf", one], cwd=cwd, capture_output=True, text=True, timeout=600)
    assert r1.returncode == 0, r1.stdout[-2000:]
    sh = str(tmp_path / "sharded.vcf")
    lib = os.path.join(ROOT, "tests", "native", "build", "libpm_cpu_driver.so")
    os.environ["PM_BLOCK_STATS"] = "1"
    try:
        r2 = run_sharded(cwd, bargs + ["--out_vcf", sh], world, lib=lib)
    finally:
        del os.environ["PM_BLOCK_STATS"]
    assert r2.returncode == 0, r2.stdout[-3000:] + r2.stderr[-3000:]
    assert vcf_body(sh) == vcf_body(one)
    assert summary_lines(r2.stdout) == summary_lines(r1.stdout) and summary_lines(r1.stdout)
    # blocks each rank read, per section, against the index
    got = {}
    for m in re.finditer(r"PM_BLOCK_STATS shard (\d+) section (\S+): blocks read (\d+)", r2.stderr):
        got[(int(m.group(1)), m.group(2))] = int(m.group(3))
    secs = blocks.read_sections(pmb)
    index = blocks.read_index(pmb)
    checked = 0
    for s, (label, mp) in enumerate(secs):
        ents = [e for e in index if e["section"] == s]
        for R in range(world):
            if (R, label) not in got:
                continue   # section not analysed (--chr2process)
            lo, hi = mp * R // world, (mp * (R + 1) // world if R < world - 1 else 1 << 62)
            want = sum(1 for e in ents if e["last_pos"] >= lo and e["first_pos"] < hi)
            assert got[(R, label)] == want, (R, label, got[(R, label)], want, lo, hi)
            checked += 1
    assert checked >= world
    if case == "example":   # the later ranks read a fraction of the section, not its whole prefix
        assert got[(world - 1, "1")] <= len(index) // world + 1


@pytest.mark.parametrize("case,world", [("example", 2), ("ragged", 2), ("quad_chrX", 2), ("late_chrX", 2),
                                        ("quad_chrX", 3), ("multi_all", 3), ("multi_chr2process", 2)])
def test_sharded_driver_matches_one_process_gloo(cpu_driver, tmp_path, case, world):
    """The multi-process driver (polymutt_amd/launch.py: contiguous position range per rank, one exchange per
    section over gloo) on the CPU oracle writes the same VCF and section summaries as one process."""
    cwd, args = _sharded_case(tmp_path, case)
    one = str(tmp_path / "one.vcf")
    r1 = subprocess.run([cpu_driver] + args + ["--out_vcf", one], cwd=cwd, capture_output=True, text=True, timeout=600)
    assert r1.returncode == 0, r1.stdout[-2000:]
    sh = str(tmp_path / "sharded.vcf")
    lib = os.path.join(ROOT, "tests", "native", "build", "libpm_cpu_driver.so")
    r2 = run_sharded(cwd, args + ["--out_vcf", sh], world, lib=lib)
    assert r2.returncode == 0, r2.stdout[-3000:] + r2.stderr[-3000:]
    assert vcf_body(sh) == vcf_body(one)
    assert summary_lines(r2.stdout) == summary_lines(r1.stdout) and summary_lines(r1.stdout)
    assert not [f for f in os.listdir(os.path.dirname(sh)) if ".part" in f]   # shard files merged and removed
    assert ("first record re-run" in r2.stderr) == (case == "late_chrX"), r2.stderr[-2000:]


@pytest.mark.parametrize("case", ["example", "late_chrX"])
def test_sharded_protocol_world_one_gloo(cpu_driver, tmp_path, monkeypatch, case):
    """PM_COLLECTIVE=gloo at world 1: the sharded protocol (part file, per-section all-gather, merge) over one rank
    writes the same VCF and summaries as the plain one-process run (the CPU twin of the RCCL world-1 GPU test)."""
    cwd, args = _sharded_case(tmp_path, case)
    one = str(tmp_path / "one.vcf")
    r1 = subprocess.run([cpu_driver] + args + ["--out_vcf", one], cwd=cwd, capture_output=True, text=True, timeout=600)
    assert r1.returncode == 0, r1.stdout[-2000:]
    sh = str(tmp_path / "w1.vcf")
    lib = os.path.join(ROOT, "tests", "native", "build", "libpm_cpu_driver.so")
    monkeypatch.setenv("PM_COLLECTIVE", "gloo")
    r2 = run_sharded(cwd, args + ["--out_vcf", sh], 1, lib=lib)
    assert r2.returncode == 0, r2.stdout[-3000:] + r2.stderr[-3000:]
    assert "collective backend gloo, world 1" in r2.stderr
    assert vcf_body(sh) == vcf_body(one)
    assert summary_lines(r2.stdout) == summary_lines(r1.stdout) and summary_lines(r1.stdout)


@pytest.mark.parametrize("case,world", [("golden", 2), ("golden", 3), ("edits", 2), ("nodata", 2), ("nodata", 3),
                                        ("empty_rank", 3)])
def test_sharded_vcf_input_matches_one_process_gloo(cpu_driver, tmp_path, case, world):
    """--in_vcf over several processes (a byte slice of the records per rank, vcf_input.cpp) writes the same VCF as
    one process: gzip and plain input, the record-kind edits, and records without data at every rank's start
    (printed with the previous computed record's state, PedVCF.cpp:113-122, handed over from an earlier rank --
    two ranks back when the rank between has no data at all)."""
    from vcf_edits import write_edited_vcf, write_nodata_vcf
    if case == "golden":
        src = os.path.join(EXAMPLE, "testvcf.in.vcf.gz")
    else:
        src = str(tmp_path / "in.vcf")
        if case == "edits":
            write_edited_vcf(src)
        elif case == "nodata":
            write_nodata_vcf(src, worlds=(2, 3))
        else:
            write_nodata_vcf(src, worlds=(3,), empty_rank=(1, 3))
    args = ["-p", "test.ped", "-d", "test.dat", "--in_vcf", src]
    one = str(tmp_path / "one.vcf")
    r1 = subprocess.run([cpu_driver] + args + ["--out_vcf", one], cwd=EXAMPLE, capture_output=True, text=True, timeout=600)
    assert r1.returncode == 0, r1.stdout[-2000:] + r1.stderr[-2000:]
    sh = str(tmp_path / "sharded.vcf")
    lib = os.path.join(ROOT, "tests", "native", "build", "libpm_cpu_driver.so")
    r2 = run_sharded(EXAMPLE, args + ["--out_vcf", sh], world, lib=lib)
    assert r2.returncode == 0, r2.stdout[-3000:] + r2.stderr[-3000:]
    assert vcf_body(sh) == vcf_body(one)
    assert len(vcf_body(one)) > 8000
    assert not [f for f in os.listdir(os.path.dirname(sh)) if ".part" in f]
    if case == "golden":
        import gzip
        gold = gzip.open(os.path.join(EXAMPLE, "testvcf.out.vcf.body.gz"), "rt").read().splitlines()
        assert vcf_body(sh)[1:] == gold[1:]
    elif case != "edits":   # the first three records have no DP key and precede the first that has one: the reference writes each
        # record at once, before DP's FORMAT index is known (FamilyLikelihoodSeq_VCF.cpp:311-314, 470, 512), so they
        # print DP=0 and '.' per sample although later records of the same batch find the index
        recs = [l.split("\t") for l in vcf_body(one)[1:]]
        for k, c in enumerate(recs[:4]):
            dp_info = c[7].split(";")[-1]
            dps = {x.split(":")[2] for x in c[9:]}
            if k < 3:
                assert dp_info == "DP=0" and dps == {"."}, (k, c[7], dps)
            else:
                assert dp_info != "DP=0" and "." not in dps, (k, c[7], dps)


@pytest.mark.parametrize("shape,n_shapes", [("ext10", 1), ("roof", 1), ("roof2", 1), ("extmix", 5)])
def test_schedule_compiler_builds_every_class(tmp_path, shape, n_shapes):
    """The Elston-Stewart schedule compiler (polymutt_amd/csrc/es_jit.h) generates the hoisting kernel of a
    pedigree's extended families for every chromosome class and hipRTC compiles it for gfx950 (no device needed);
    families of one shape share one device function, and a mixed pedigree file (extmix: five 8-12-member shapes)
    gets one function per shape behind the kernel's shape switch; --denovo engines get the wave-cooperative variant."""
    exe = os.path.join(ROOT, "tests", "native", "build", "jit_check")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "polymutt_amd"), "../tests/native/build/jit_check"], check=True)
    pm.synth_write_dataset(str(tmp_path), shape, 5, 1, 3)
    r = subprocess.run([exe, str(tmp_path / "test.dat"), str(tmp_path / "test.ped"), "--emit", str(tmp_path / "k.hip")],
                       capture_output=True, text=True, timeout=300, env=dict(os.environ, PM_JIT_LAYOUT="1"))
    assert r.returncode == 0, r.stdout + r.stderr
    # the static lane occupancy per generated function (useful FP64 element-ops / issued lane slots), in (0, 1]
    occ = [l.split() for l in r.stderr.splitlines() if l.startswith("occupancy")]
    assert occ and all(0.0 < float(l[-1]) <= 1.0 for l in occ), r.stderr[-2000:]
    lines = [l.split() for l in r.stdout.splitlines() if l.startswith("class")]
    assert [int(l[1]) for l in lines] == [0, 1, 2, 3] * 3   # bi-allelic engines, --denovo (grouped tasks, then all)
    assert all(int(l[3]) == n_shapes and int(l[5]) == 5 and int(l[9]) > 0 for l in lines), r.stdout   # shapes, 5 families
    src = (tmp_path / "k.hip").read_text()
    assert "es_hoist_jit" in src and "asm" not in src
    assert all(f"fam{i}(" in src for i in range(n_shapes)) and f"fam{n_shapes}(" not in src
    # --denovo kernels: the grouped-tasks-only kernel (lines 4-7) needs no larger a workspace slice than the one with
    # the whole 10-state / top variants (lines 8-11); per (item, family) the leaf prefix + 10-state rest does the
    # whole 10-state peel's operations or fewer (founder sparsity), and the top rest + leaf the top variant's
    def field(l, name):
        return int(l[l.index(name) + 1])
    for g, f in zip(lines[4:8], lines[8:12]):
        assert field(g, "ws") <= field(f, "ws"), (g, f)
        ops = [float(x) for x in f[f.index("ops") + 1:]]   # bi-allelic, 10-state, top, leaf, rest, top rest
        assert ops[3] + ops[4] <= ops[1] + 1e-9 and ops[3] + ops[5] <= ops[2] + 1e-9, f
