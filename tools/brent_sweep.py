"""Sweep Brent-kernel geometries (threads x families-per-lane) on the quad workload (experiment tool)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import polymutt_amd as pm  # noqa: E402

nfam = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
variants = sys.argv[2].split(";") if len(sys.argv) > 2 else ["256,4", "512,2", "1024,1", "128,8", "64,16", "1024,2"]
B = 32768
ped = bench.quad_pedigree(pm, nfam, 2)
for v in variants:
    os.environ["PM_BRENT_TS"] = v
    for exact in [int(x) for x in os.environ.get("PM_SWEEP_NUMERICS", "0,2").split(",")]:
        eng = pm.Engine(ped, pm.Params.defaults(numerics=exact), max_batch=B)
        d_pl, d_dm, d_ref = eng.alloc(B * ped.n_person * 10), eng.alloc(B * ped.n_person * 4), eng.alloc(B)
        eng.synth(B, 7, 0, d_pl, d_dm, d_ref)
        eng.run_device(B, d_pl, d_dm, d_ref); eng.sync()
        eng.kernel_stats(reset=True)
        t0 = time.perf_counter()
        for _ in range(4):
            eng.run_device(B, d_pl, d_dm, d_ref)
            eng.sync()
        dt = time.perf_counter() - t0
        ks = eng.kernel_stats()
        print(f"T,S={v:8s} numerics={exact}  brent {ks.kernel_ms/4:8.3f} ms/step  total {dt/4*1e3:8.3f} ms/step  "
              f"sites/s {4*B/dt:12.0f}  evals/item {ks.evals/max(1,ks.items):.2f}", flush=True)
        for p in (d_pl, d_dm, d_ref):
            eng.free(p)
        eng.close()
