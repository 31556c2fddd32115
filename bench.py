#!/usr/bin/env python3
"""bench.py -- headline benchmark of the MI355X polyMutt engine.

Metric (BASELINE.json): sites/s for the whole node, 1000 nuclear quad families, synthetic GLF sites
(SURVEY.md 8(d) recipe, generated on the device), plus achieved HBM GB/s and the FP64 roofline of the
dominant kernel (k_brent).  A "step" = one pass of the full per-site path (read stats, filters,
monomorphism, 3(+3) Brent-optimised allele configurations, model selection, genotype posteriors)
over one batch of sites already resident in HBM.

Multi-GPU: one process per GPU (torchrun); sites are sharded (weak scaling, no data-path collective);
the section summary counters are combined with one RCCL all-reduce, as the north star prescribes.

cpu_baseline: the reference itself (oracle/_ref/pm_ref, built from /root/reference sources; it travels
to the GPU box as a prebuilt binary) on a bounded sample of the same synthetic workload written as GLF
files, timed on the host cores -- rank 0, N=1 only.
"""
import argparse
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

FP64_PEAK_TFLOPS = 78.6       # MI355X FP64 vector (FMA counted as 2), datasheet
FP64_NONFMA_TFLOPS = 39.3     # issue rate of non-fused FP64 mul/add (the engine issues no FMA: parity)
HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--families", type=int, default=1000)
    ap.add_argument("--kids", type=int, default=2)
    ap.add_argument("--batch", type=int, default=65536, help="sites per step per GPU")
    ap.add_argument("--pool", type=int, default=2, help="distinct resident batches cycled by the steps")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--cpu-sites", type=int, default=2000)
    ap.add_argument("--cpu-threads", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def quad_pedigree(pm, nfam, kids):
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


def cpu_baseline(args):
    """Reference binary (or the CPU port) on a bounded GLF sample of the same workload."""
    import polymutt_amd as pm
    ref_bin = os.path.join(ROOT, "oracle", "_ref", "pm_ref")
    port_bin = os.path.join(ROOT, "tests", "native", "build", "cpu_polymutt")
    if os.path.exists(ref_bin):
        exe, kind = ref_bin, "reference"
    elif os.path.exists(port_bin):
        exe, kind = port_bin, "port"
    else:
        return None
    tmp = tempfile.mkdtemp(prefix="pm_cpu_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        shape = "quad" if args.kids == 2 else "trio"
        pm.synth_write_dataset(tmp, shape, args.families, args.cpu_sites, args.seed)
        cmd = [exe, "-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--out_vcf", "out.vcf",
               "--nthreads", str(args.cpu_threads)]
        t0 = time.perf_counter()
        r = subprocess.run(cmd, cwd=tmp, capture_output=True, text=True, timeout=600)
        dt = time.perf_counter() - t0
        if r.returncode != 0:
            return {"error": r.stdout[-500:]}
        return {"value": args.cpu_sites / dt, "unit": "sites/s", "cores": args.cpu_threads, "kind": kind,
                "sample": f"{args.families} synthetic {shape} families x {args.cpu_sites} sites written as GLF (seed "
                          f"{args.seed}), end-to-end wall time incl. GLF ingest, --nthreads {args.cpu_threads}",
                "seconds": dt}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    import polymutt_amd as pm

    ped = quad_pedigree(pm, args.families, args.kids)
    B, P = args.batch, args.pool
    eng = pm.Engine(ped, pm.Params.defaults(), device=local, max_batch=B)
    npers = ped.n_person
    bufs = []
    for p in range(P):
        d_pl, d_dm, d_ref = eng.alloc(B * npers * 10), eng.alloc(B * npers * 4), eng.alloc(B)
        eng.synth(B, args.seed, (rank * P + p) * B, d_pl, d_dm, d_ref)
        bufs.append((d_pl, d_dm, d_ref))

    def step(i):
        d_pl, d_dm, d_ref = bufs[i % P]
        eng.run_device(B, d_pl, d_dm, d_ref)
        eng.sync()

    def barrier():
        if dist is not None:
            dist.barrier()

    for i in range(args.warmup):
        step(i)
    eng.begin_section(pm.PM_CHR_AUTO)   # counters of the timed region only
    eng.kernel_stats(reset=True)
    barrier()
    eng.sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    eng.sync()
    barrier()
    elapsed = time.perf_counter() - t0
    ks = eng.kernel_stats()
    counters = eng.counters().as_array()
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        c = torch.tensor(counters, dtype=torch.int64, device="cuda")
        dist.all_reduce(c, op=dist.ReduceOp.SUM)   # the single RCCL all-reduce of the section counters
        counters = c.cpu().numpy()

    total_sites = B * args.steps * world
    value = total_sites / elapsed
    # dominant kernel roofline (SURVEY 8(d) algorithmic op count, log10 counted as 1 op)
    nf, K = args.families, args.kids
    ops = ks.evals * (19 * nf + 17) + ks.items * nf * (18 + 36 * K)
    kern_s = ks.kernel_ms * 1e-3
    achieved = ops / kern_s / 1e12 if kern_s > 0 else 0.0
    b_site = 14 * npers + 1
    if rank == 0:
        out = {
            "metric": "sites/sec (whole node) + achieved HBM GB/s, 1000 quad families",
            "value": value, "unit": "sites/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": f"{nf} nuclear families (2 parents + {K} kids), synthetic GLF sites per SURVEY 8(d), "
                                   f"dense blocks resident in HBM", "families": nf, "persons": npers,
                       "sites_per_step_per_gpu": B, "distinct_sites_per_gpu": B * P, "parallelism": f"site-shard x{world}"},
            "roofline": {"bound": "fp64-valu", "kernel": "k_brent", "achieved": achieved, "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": achieved / FP64_PEAK_TFLOPS,
                         "frac_of_nonfma_issue_peak": achieved / FP64_NONFMA_TFLOPS, "traffic": None,
                         "launches": ks.launches, "kernel_ms_total": ks.kernel_ms,
                         "avg_launch_ms": ks.kernel_ms / max(1, ks.launches), "evals": ks.evals, "items": ks.items,
                         "log10_per_s": ks.evals * nf / kern_s if kern_s > 0 else 0.0,
                         "ops_per_site": ops / max(1, ks.sites)},
            "hbm": {"algorithmic_bytes_per_site": b_site, "achieved_GBs": value * b_site / 1e9 / world,
                    "peak_GBs": HBM_PEAK_GBS, "frac": value * b_site / 1e9 / world / HBM_PEAK_GBS},
            "counters": {"sites": int(counters[:5].sum()), "homo_ref": int(counters[9]),
                         "transitions": int(counters[10]), "transversions": int(counters[11]),
                         "nocall": int(counters[15])},
        }
        if world == 1 and not args.no_cpu_baseline:
            cb = cpu_baseline(args)
            out["cpu_baseline"] = cb
            if cb and "value" in cb:
                out["speedup_vs_cpu_baseline"] = value / cb["value"]
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    for d in bufs:
        for p in d:
            eng.free(p)
    eng.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
