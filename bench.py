#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X polyMutt engine.

Metric (BASELINE.json): sites/s for the whole node, 1000 nuclear quad families, synthetic GLF-shaped sites
(SURVEY.md 8(d) recipe, generated on the device), plus achieved HBM GB/s.  Default workload = BASELINE config 3,
the configuration the metric is quoted on: 1000 nuclear quads x 10M sites with the --denovo MutationModel
(40 steps x 262 144 sites = 10.5M sites per GPU); --no-denovo gives the plain quad model.  A "step" = one pass of the
full per-site path (read stats, filters, monomorphism, 3(+3) Brent-optimised allele configurations, model
selection, de novo LR with --denovo, genotype posteriors, allele balance) over one batch of sites already
resident in HBM.  Consecutive batches go to --engines engine instances (default 3), each with its own HIP
stream and work buffers, so one batch's HBM-bound k_prep and small tail launches overlap another batch's
FP64-bound Brent kernel (the host waits on an engine only before giving it its next batch).

Roofline: the dominant kernel is k_brent (the Brent allele-frequency maximisation), which is FP64-VALU bound
(SURVEY 8(d)).  `roofline` is that FP64 roofline: the SURVEY 8(d) algorithmic op count (nuclear families:
evals x (19 nFam + 17) + items x nFam x (18 + 36 K); extended families: the per-evaluation peel op counts of
their schedules) over k_brent's own kernel time, against the 39.3 T non-FMA FP64 ops/s of the spec (78.6
TFLOP/s FMA-counted).  The kernel time comes from a one-engine calibration pass after the timed region (HIP
events around every k_brent launch on that engine's stream; with one engine nothing overlaps a launch, so the
events agree with rocprofv3's kernel records -- profiles/r02*_kernel_stats_1engine.csv).  `achieved_wall`
is the timed region's ops per wall second.  `roofline_hbm` is the HBM figure BASELINE.json asks for
(algorithmic bytes = each launch reads the PL block of every site it touches once), with `traffic` = the
PMC-measured HBM bytes per k_brent dispatch from the committed rocprofv3 passes under profiles/.

Multi-GPU: one process per GPU; sites are sharded (weak scaling, no data-path collective); the section
summary counters are combined with one RCCL all-reduce (polymutt_amd/shard.py).  `--gpus N` with N > 1 and
no WORLD_SIZE in the environment starts `torch.distributed.run --nproc-per-node N` on this script as a child
process (before anything touches the GPU) and relays its exit code; the workers check WORLD_SIZE == N and
the line records `rccl_world`, the world size the counter all-reduce actually ran over.  `--dry-run` runs the
same launcher and collectives over gloo with no engine (tests/test_cpu_host.py).

cpu_baseline: the clean-room CPU restatement of the reference path (tests/native/build/cpu_polymutt: the
product host driver over the oracle, with the reference's OpenMP sections over the allele configurations) on
bounded GLF slices of the same workload, timed on the box's host cores at 1 thread and at the box's CPU share,
best of 3 -- rank 0, N=1 only.  Two slice sizes give the steady per-site rate with start-up (pedigree load,
GLF opens) subtracted.  The reference's own objects never travel to the box (license.txt:1);
tools/cpu_calibrate.py measures the reference against the restatement in the build container
(profiles/r03_cpu_calibration.json) and the line carries that ratio and the implied reference rate.
"""
import argparse
import glob
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md (spec)
CPU_SHARE = 16                # host threads a GPU box grants one GPU (OMP_NUM_THREADS there)
FP64_PEAK_TFLOPS = 78.6       # MI355X FP64 vector, FMA counted as 2 (spec)
FP64_NONFMA_TOPS = 39.3       # mul/add issue rate = half the FMA-counted peak (profiles/*_fp64_peak.json measures it)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one process each); N > 1 without WORLD_SIZE starts torch.distributed.run itself")
    ap.add_argument("--rccl", action="store_true",
                    help="initialise the RCCL (nccl) process group and run the counter all-reduce on the device even at "
                         "one rank (exercises the multi-GPU collective path on a one-GPU box)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher + collectives only (gloo, no engine, no GPU): checks the multi-process path")
    ap.add_argument("--steps", type=int, default=400)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--families", type=int, default=1000)
    ap.add_argument("--shape", choices=["quad", "trio", "ext10", "extmix", "mixed"], default="quad",
                    help="quad/trio: BASELINE configs 2-3; ext10: config 4 (3-generation pedigrees, ES peeling), one "
                         "10-member shape; extmix: config 4 at its stated 8-12-member range (ext10, roof, roof2, ext12, "
                         "ext11 round-robin); mixed: trios and quads (config 5 with --vcf)")
    ap.add_argument("--vcf", action="store_true", help="BASELINE config 5: the --in_vcf engine mode (one Brent per site)")
    ap.add_argument("--denovo", dest="denovo", action="store_true", default=True,
                    help="BASELINE config 3: --denovo MutationModel (default)")
    ap.add_argument("--no-denovo", dest="denovo", action="store_false", help="plain (non-de-novo) quad model")
    ap.add_argument("--batch", type=int, default=262144, help="sites per step per GPU (40 x 262 144 = 10.5 M sites)")
    ap.add_argument("--pool", type=int, default=4, help="distinct resident batches cycled by the steps")
    ap.add_argument("--engines", type=int, default=3,
                    help="engine instances (each with its own HIP stream and work buffers) taking consecutive batches: "
                         "one batch's HBM-bound k_prep overlaps the previous batch's FP64-bound Brent kernel")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--cpu-sites", type=int, nargs=2, default=[500, 2500],
                    help="the two GLF slice sizes of the cpu_baseline (steady rate = their difference over the time difference)")
    ap.add_argument("--cpu-reps", type=int, default=3, help="cpu_baseline: best of this many runs per slice and thread count")
    ap.add_argument("--calib-steps", type=int, default=12,
                    help="one-engine steps after the timed region that give k_brent's own kernel time")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-inputs", action="store_true",
                    help="PCIe-inclusive variant: blocks start in host memory and results return to the host "
                         "(pm_engine_run); never the headline value")
    args = ap.parse_args()
    if args.vcf:
        args.denovo = False   # the VCF path has no de novo model (PedVCF.cpp)
    return args


def nuclear_pedigree(pm, nfam, kids):
    size = 2 + kids
    n = nfam * size
    sex = np.zeros(n, np.int8)
    isf = np.zeros(n, np.int8)
    fa = np.full(n, -1, np.int32)
    mo = np.full(n, -1, np.int32)
    for f in range(nfam):
        b = f * size
        sex[b], sex[b + 1] = 1, 2
        isf[b] = isf[b + 1] = 1
        for k in range(kids):
            sex[b + 2 + k] = 1 + (k % 2)
            fa[b + 2 + k], mo[b + 2 + k] = b, b + 1
    kind = np.full(nfam, pm.FAM_NUCLEAR if kids > 0 else pm.FAM_FOUNDERS, np.int32)
    return pm.pedigree_from_arrays(np.full(nfam, size), np.full(nfam, 2), kind, sex, isf, fa, mo)


quad_pedigree = nuclear_pedigree   # used by __graft_entry__.smoke()


def cpu_model():
    try:
        for l in open("/proc/cpuinfo"):
            if l.startswith("model name"):
                return l.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_calibration(args):
    """The reference-vs-restatement ratios tools/cpu_calibrate.py measured in the build container on the default
    workload, per thread count (profiles/r*_cpu_calibration.json), or None."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_cpu_calibration.json")))
    if not files or (args.shape, args.families, args.denovo, args.vcf) != ("quad", 1000, True, False):
        return None
    d = json.load(open(files[-1]))
    if "reference_over_port" not in d:
        return None
    return {"file": os.path.basename(files[-1]), "reference_over_port": d["reference_over_port"],
            "build_container_nproc": d["nproc"]}


def cpu_baseline(args):
    """The clean-room CPU restatement (product host driver + the oracle, with the reference's OpenMP structure:
    `omp parallel sections` over the allele configurations, main.cpp:439-536, and the family loop's `parallel for`,
    FamilyLikelihoodSeq.cpp:225) on two bounded GLF slices of the same workload, at 1 thread and at the box's CPU
    share, best of --cpu-reps runs each; value = the steady per-site rate (slice difference over time difference),
    so start-up (pedigree load, one GLF open per person) does not inflate the GPU/CPU ratio."""
    import polymutt_amd as pm
    exe = os.path.join(ROOT, "tests", "native", "build", "cpu_polymutt")
    if not os.path.exists(exe):
        return None
    s1, s2 = sorted(args.cpu_sites)
    tmp = tempfile.mkdtemp(prefix="pm_cpu_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        dirs = {}
        for s in (s1, s2):
            dirs[s] = os.path.join(tmp, str(s))
            pm.synth_write_dataset(dirs[s], args.shape, args.families, s, args.seed)
        runs = {}
        for th in (1, CPU_SHARE):
            secs = []
            for s in (s1, s2):
                best = None
                for _ in range(args.cpu_reps):
                    cmd = [exe, "-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--out_vcf", "out.vcf",
                           "--nthreads", str(th)] + (["--denovo"] if args.denovo else [])
                    t0 = time.perf_counter()
                    r = subprocess.run(cmd, cwd=dirs[s], capture_output=True, text=True, timeout=900,
                                       env=dict(os.environ, OMP_NUM_THREADS=str(th)))
                    dt = time.perf_counter() - t0
                    if r.returncode != 0:
                        return {"error": r.stdout[-500:]}
                    best = dt if best is None else min(best, dt)
                secs.append(best)
            steady = (s2 - s1) / (secs[1] - secs[0]) if secs[1] > secs[0] else s2 / secs[1]
            runs[th] = {"value": steady, "seconds_best": secs, "end_to_end": s2 / secs[1]}
        th_best = max(runs, key=lambda t: runs[t]["value"])
        out = {"value": runs[th_best]["value"], "unit": "sites/s", "cores": th_best, "kind": "port",
               "value_1thread": runs[1]["value"], "value_best": runs[th_best]["value"], "threads_best": th_best,
               "runs": {str(t): v for t, v in runs.items()}, "nproc": os.cpu_count(), "cpu_share": CPU_SHARE,
               "cpu_model": cpu_model(),
               "sample": f"{args.families} synthetic {args.shape} families (seed {args.seed}) x {s1} and x {s2} sites "
                         f"written as GLF" + (", --denovo" if args.denovo else "") + "; the restatement "
                         "(tests/native/build/cpu_polymutt, the reference's OpenMP sections) end to end incl. GLF "
                         f"ingest at 1 and {CPU_SHARE} threads, best of {args.cpu_reps}; value = ({s2} - {s1}) sites / "
                         f"(t{s2} - t{s1}) at the faster thread count"}
        cal = cpu_calibration(args)
        if cal:   # what the reference itself would do on these cores, from the build container's ratios
            ratio = cal["reference_over_port"]
            t_hi = str(max(int(k) for k in ratio))
            out["calibration"] = cal
            out["reference_equivalent_1thread"] = runs[1]["value"] * ratio["1"]
            out["reference_equivalent_best"] = max(runs[1]["value"] * ratio["1"],
                                                   runs[CPU_SHARE]["value"] * ratio[t_hi])
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def peel_ops(ped_view, n_states):
    """SURVEY 8(d) per-evaluation op count of every extended family's Elston-Stewart peel (its schedule from
    the pedigree), summed: type 1 (offspring -> parents) ns^2 (2 ns + 1), type 2 (spouse -> spouse)
    ns (2 ns + 1), type 3 (parents -> only child) 4 ns^3 + ns, founder priors ns per founder, final sum
    ns - 1 adds + 1 log10.  BA (ns = 3): 63 / 21 / 111, as SURVEY 8(d) lists them."""
    import polymutt_amd as pm
    ns = n_states
    cost = {1: ns * ns * (2 * ns + 1), 2: ns * (2 * ns + 1), 3: 4 * ns ** 3 + ns}
    v = ped_view
    kinds = np.ctypeslib.as_array(v.fam_kind, shape=(v.n_fam,))
    founders = np.ctypeslib.as_array(v.fam_founders, shape=(v.n_fam,))
    if not v.peel_start:
        return 0, 0
    ps = np.ctypeslib.as_array(v.peel_start, shape=(v.n_fam + 1,))
    total, n_ext = 0, 0
    for f in range(v.n_fam):
        if kinds[f] != pm.FAM_EXTENDED:
            continue
        n_ext += 1
        total += sum(cost[v.steps[i].type] for i in range(ps[f], ps[f + 1])) + ns * int(founders[f]) + ns
    return total, n_ext


def ep_eval_ops(ped_view):
    """FP64 operations k_brent's EP instantiation executes per objective evaluation for the extended families (the
    polynomial form, es_poly_eval): t = f / g or g / f (2), D Horner steps (multiply + add), D multiplies for the
    base power, one for the product, and the (mantissa, exponent) product (2): 3 D + 5 per family, D = 2 x founders
    on autosomes."""
    import polymutt_amd as pm
    v = ped_view
    kinds = np.ctypeslib.as_array(v.fam_kind, shape=(v.n_fam,))
    founders = np.ctypeslib.as_array(v.fam_founders, shape=(v.n_fam,))
    return int(sum(3 * 2 * int(founders[f]) + 5 for f in range(v.n_fam) if kinds[f] == pm.FAM_EXTENDED))


def pmc_traffic():
    """HBM bytes per k_brent dispatch from the newest committed PMC summary (profiles/rNN_pmc.json: the default
    workload on one engine, tools/profile_round.sh)."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json")))
    if not files:
        return None, None
    d = json.load(open(files[-1]))
    # the source is stamped with the tree revision its PMC passes ran on (the summary's "revision", else "unknown"),
    # so a traffic figure from an older kernel shows as such
    src = os.path.basename(files[-1]) + "@" + str(d.get("revision", "unknown"))[:20]
    for k, v in d.items():
        if k.startswith("k_brent") and isinstance(v, dict) and "hbm_read_bytes_per_dispatch" in v:
            return v["hbm_read_bytes_per_dispatch"] + v.get("hbm_write_bytes_per_dispatch", 0.0), src
    return None, src


def phase_split(st):
    """k_brent's in-kernel hoisting / evaluation split (PM_PHASE_TIMING=1 at engine creation; else None): wave
    time per item in each phase, from lane 0's 100 MHz clock."""
    if not st.timed_items:
        return None
    h, e = st.hoist_wave_ns / st.timed_items, st.eval_wave_ns / st.timed_items
    return {"hoist_us_per_item": h / 1e3, "eval_us_per_item": e / 1e3, "hoist_frac": h / (h + e) if h + e else 0.0,
            "timed_items": st.timed_items}


def measured_fp64_peak():
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_fp64_peak.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    rates = [d[k] for k in ("v_mul_f64_Tops", "v_add_f64_Tops") if k in d]
    return max(rates) if rates else None   # the faster of mul/add: the conservative (larger) peak


def launch_workers(args):
    """`bench.py --gpus N` (N > 1) run directly: one worker process per GPU under torch.distributed.run, started
    as a child before this process touches the GPU; rank 0's JSON line reaches our stdout unchanged."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=dict(os.environ, PYTHONUNBUFFERED="1")).returncode


def dry_run(args, world, rank):
    """The multi-process skeleton without an engine: gloo process group, barrier, counter all-reduce and
    max-over-ranks timing, exactly as the GPU path does them; one JSON line from rank 0."""
    import torch.distributed as dist
    from polymutt_amd.shard import allreduce_counters, max_over_ranks
    if world > 1:
        dist.init_process_group("gloo")
        dist.barrier()
    t0 = time.perf_counter()
    counters = allreduce_counters(np.full(16, rank + 1, np.int64))
    elapsed = max_over_ranks(time.perf_counter() - t0)
    rw = dist.get_world_size() if dist.is_initialized() else 1
    if rank == 0:
        print(json.dumps({"metric": "dry-run", "value": None, "n_gpus": world, "rccl_world": rw,
                          "backend": dist.get_backend() if dist.is_initialized() else None,
                          "counter_sum": int(counters[0]), "elapsed": elapsed}), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:
        sys.exit(launch_workers(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.dry_run:
        return dry_run(args, world, rank)
    dev = None
    if world > 1 or args.rccl:
        import torch
        import torch.distributed as dist
        if world == 1:   # a one-rank group of our own (no launcher): loopback rendezvous on a free port
            import socket
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                os.environ.setdefault("MASTER_PORT", str(s.getsockname()[1]))
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
        dev = torch.device("cuda", local)
    import polymutt_amd as pm
    from polymutt_amd.shard import allreduce_counters, max_over_ranks

    kids = {"quad": 2, "trio": 1, "mixed": 2, "ext10": 2, "extmix": 2}[args.shape]
    if args.shape in ("quad", "trio"):
        ped = nuclear_pedigree(pm, args.families, kids)
        ped_keep = None
    else:   # pedigrees with ES schedules come from the native loader (synthetic .ped written once)
        tmpd = tempfile.mkdtemp(prefix="pm_ped_", dir=os.environ.get("TMPDIR", "/tmp"))
        pm.synth_write_dataset(tmpd, args.shape, args.families, 1, args.seed)
        ped_keep = pm.Pedigree(os.path.join(tmpd, "test.dat"), os.path.join(tmpd, "test.ped"))
        shutil.rmtree(tmpd, ignore_errors=True)
        ped = ped_keep.view
    B, P = args.batch, args.pool
    params = pm.Params.defaults(denovo=1 if args.denovo else 0, vcf_mode=1 if args.vcf else 0)
    engines = [pm.Engine(ped, params, device=local, max_batch=B) for _ in range(max(1, args.engines))]
    eng = engines[0]
    npers = ped.n_person
    bufs = []
    for p in range(P):   # this rank's shard of the synthetic site stream (weak scaling)
        d_pl, d_dm, d_ref = eng.alloc(B * npers * 10), eng.alloc(B * npers * 4), eng.alloc(B)
        eng.synth(B, args.seed, (rank * P + p) * B, d_pl, d_dm, d_ref)
        if args.vcf:   # (ref, alt = transition) per site, as a biallelic VCF record carries it
            href = np.empty(B, np.uint8)
            eng.to_host(href, d_ref, B)
            ts = np.array([0, 3, 4, 1, 2], np.uint8)
            href = (href | (ts[href] << 4)).astype(np.uint8)
            eng.free(d_ref)
            d_ref = eng.alloc(B)
            eng.to_device(d_ref, href, B)
        bufs.append((d_pl, d_dm, d_ref))

    host = None
    if args.host_inputs:   # the same sites as person-major host arrays (pageable), pm_engine_run's layout
        host = []
        for p in range(P):
            hpl, hdm, href = pm.synth_block_host(ped, B, args.seed, (rank * P + p) * B)
            if args.vcf:
                eng.to_host(href, bufs[p][2], B)
            host.append((hpl, hdm, href))

    pending = [False] * len(engines)

    def step(i):
        if host is not None:
            eng.run(*host[i % P])   # H2D inputs, pipeline, D2H results + genotype rows
            return
        d_pl, d_dm, d_ref = bufs[i % P]
        k = i % len(engines)
        if pending[k]:
            engines[k].sync()   # this engine's previous batch (its stats, Brent status); the others keep running
        engines[k].run_device(B, d_pl, d_dm, d_ref)
        pending[k] = True

    def drain():
        for k, e in enumerate(engines):
            if pending[k]:
                e.sync()
                pending[k] = False

    def barrier():
        if dev is not None:
            import torch.distributed as dist
            dist.barrier()

    for i in range(args.warmup):
        step(i)
    drain()
    for e in engines:
        e.begin_section(pm.PM_CHR_AUTO)   # counters of the timed region only
        e.kernel_stats(reset=True)
    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    drain()
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dev)
    kss = [e.kernel_stats() for e in engines]
    ks = type(kss[0])()
    for f, _ in ks._fields_:
        setattr(ks, f, sum(getattr(x, f) for x in kss))
    counters = allreduce_counters(sum(e.counters().as_array() for e in engines), dev)   # the single RCCL all-reduce
    if dev is not None:
        import torch.distributed as dist
        rccl_world, backend = dist.get_world_size(), dist.get_backend()
    else:
        rccl_world, backend = 1, None

    total_sites = B * args.steps * world
    value = total_sites / elapsed
    nf, K = args.families, kids
    # SURVEY 8(d) algorithmic FP64 op count of k_brent's work (log10 counted as 1 op)
    ext_ops, n_ext = peel_ops(ped, 10 if args.denovo else 3)
    n_nuc = nf - n_ext
    kid_sum = int((np.diff(np.ctypeslib.as_array(ped.fam_start, shape=(ped.n_fam + 1,))) - 2).clip(0).sum()) if n_nuc else 0
    if n_ext:
        kid_sum = 0   # (ext10 / roof shapes: every family is extended)

    # extended families with the default (POLY) numerics: k_brent evaluates the hoisted polynomials, so its executed
    # operations are counted (ep_eval_ops), and the hoisting is a kernel of its own with its own roofline below
    ep = n_ext > 0
    ext_eval_ops = ep_eval_ops(ped) if ep else ext_ops

    def fused(st):   # ep_brent_jit: the peel's hoisting runs inside the Brent kernel (no hoisting launches)
        return ep and st.es_hoist_launches == 0 and st.es_hoist_ops > 0

    def brent_ops(st):
        o = st.evals * (19 * n_nuc + 17 + ext_eval_ops) + st.items * (18 * n_nuc + 36 * kid_sum)
        return o + (st.es_hoist_ops if fused(st) else 0.0)

    ops = brent_ops(ks)
    # one-engine calibration: k_brent's own launch times (nothing overlaps a launch on a single stream)
    cal = None
    if args.calib_steps > 0 and host is None:
        e0 = engines[0]
        e0.kernel_stats(reset=True)
        for i in range(args.calib_steps):
            e0.run_device(B, *bufs[i % P])
            e0.sync()
        cal = e0.kernel_stats()
    ref_st = cal if cal is not None else ks
    kern_s = ref_st.kernel_ms * 1e-3
    launches = max(1, ref_st.launches)
    avg_launch_s = kern_s / launches
    ops_launch = brent_ops(ref_st) / launches
    achieved_tops = ops_launch / avg_launch_s / 1e12 if kern_s > 0 else 0.0
    peak_meas = measured_fp64_peak()
    # k_brent algorithmic bytes: every launch reads the PL block (nPerson x 10 B) of each site it touches once
    alg_bytes_launch = ref_st.site_visits * npers * 10 / launches
    achieved_gbs = alg_bytes_launch / avg_launch_s / 1e9 if kern_s > 0 else 0.0
    default_workload = (args.shape, args.families, args.denovo, args.vcf) == ("quad", 1000, True, False)
    traffic, pmc_file = pmc_traffic() if default_workload else (None, None)   # the PMC passes profile the default workload
    b_site = 14 * npers + 1
    if rank == 0:
        out = {
            "metric": "sites/sec (whole node) + achieved HBM GB/s, 1000 quad families",
            "value": value, "unit": "sites/s", "n_gpus": world, "rccl_world": rccl_world, "collective_backend": backend,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"{nf} {args.shape} families, synthetic GLF-shaped sites per SURVEY 8(d) generated in "
                                   f"HBM" + (", --denovo" if args.denovo else "") + (", --in_vcf engine mode" if args.vcf else ""),
                       "families": nf, "persons": npers, "sites_per_step_per_gpu": B,
                       "distinct_sites_per_gpu": B * P, "parallelism": f"site-shard x{world}",
                       "inputs": "host (PCIe-inclusive)" if args.host_inputs else "HBM-resident",
                       "engines": 1 if args.host_inputs else len(engines)},
            "roofline": {"bound": "fp64-valu", "kernel": "ep_brent_jit" if fused(ref_st) else "k_brent", "achieved": achieved_tops,
                         "peak": FP64_NONFMA_TOPS,
                         "unit": "TFLOP/s (non-FMA FP64 ops)", "frac": achieved_tops / FP64_NONFMA_TOPS,
                         "traffic": traffic, "traffic_unit": "HBM bytes per k_brent dispatch (PMC)",
                         "traffic_source": pmc_file, "ops_per_launch": ops_launch, "avg_launch_ms": avg_launch_s * 1e3,
                         "launches": ref_st.launches,
                         "time_source": ("one-engine calibration pass (HIP events on the engine stream), %d steps" % args.calib_steps)
                                        if cal is not None else "timed region",
                         "achieved_wall": ops / elapsed / 1e12, "frac_wall": ops / elapsed / 1e12 / FP64_NONFMA_TOPS,
                         "peak_measured_issue_rate": peak_meas,
                         "op_model": ("executed: evals x (19 nNuc + 17 + sum over extended families of (3 D + 5)) + items x "
                                      "(18 nNuc + 36 kids) + the generated peels' hoisting operations (fused: ep_brent_jit "
                                      "hoists and runs Brent in one kernel)") if fused(ref_st) else
                                     ("executed: evals x (19 nNuc + 17 + sum over extended families of (3 D + 5)) + items x "
                                      "(18 nNuc + 36 kids); the coefficient hoisting is roofline_es_hoist") if ep else
                                     "SURVEY 8(d): evals x (19 nNuc + 17 + peel ops) + items x (18 nNuc + 36 kids)",
                         "peel_ops_per_eval": ext_ops, "ext_eval_ops": ext_eval_ops if ep else None,
                         "evals": ks.evals, "items": ks.items,
                         "phase_split": phase_split(ref_st),
                         "ops_per_site": ops / max(1, ks.sites), "log10_per_s": ks.evals * nf / elapsed},
            "roofline_hbm": {"bound": "hbm", "kernel": "k_brent", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                             "traffic_source": pmc_file, "algorithmic_bytes_per_launch": alg_bytes_launch,
                             "achieved_wall": ks.site_visits * npers * 10 / elapsed / 1e9},
            "hbm": {"algorithmic_bytes_per_site": b_site, "achieved_GBs": value * b_site / 1e9 / world,
                    "peak_GBs": HBM_PEAK_GBS, "frac": value * b_site / 1e9 / world / HBM_PEAK_GBS},
            "counters": {"sites": int(counters[:5].sum()), "homo_ref": int(counters[9]),
                         "transitions": int(counters[10]), "transversions": int(counters[11]),
                         "nocall": int(counters[15])},
        }
        if ep and not fused(ref_st):   # the EP hoisting kernel (es_hoist_wave / es_hoist_jit): ops counted by the schedule compiler
            hs = ref_st
            h_ms = hs.es_hoist_ms / max(1, hs.es_hoist_launches)
            h_ops = hs.es_hoist_ops / max(1, hs.es_hoist_launches)
            h_t = h_ops / (h_ms * 1e-3) / 1e12 if h_ms > 0 and h_ops > 0 else None
            out["roofline_es_hoist"] = {
                "bound": "fp64-valu", "kernel": "es_hoist_wave" if args.denovo else "es_hoist_jit",
                "achieved": h_t, "peak": FP64_NONFMA_TOPS, "unit": "TFLOP/s (non-FMA FP64 ops)",
                "frac": h_t / FP64_NONFMA_TOPS if h_t else None, "ops_per_launch": h_ops, "avg_launch_ms": h_ms,
                "launches": hs.es_hoist_launches, "ms_per_step": hs.es_hoist_ms / max(1, args.calib_steps),
                "op_model": "FP64 operations of the generated peel (each mul, add or fma one), per family shape and "
                            "variant, times the hoisted (item, family) pairs"}
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(args)
            out["cpu_baseline"] = cb
            if cb and "value" in cb:   # against the faster of the port and the reference-equivalent rate
                out["speedup_vs_cpu_baseline"] = value / max(cb["value"], cb.get("reference_equivalent_best", 0.0))
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    for d in bufs:
        for p in d:
            eng.free(p)
    for e in engines:
        e.close()
    if dev is not None:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
