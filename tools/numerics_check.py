"""Compare the engine's numerics modes against the CPU oracle on a synthetic workload (experiment tool):
minimiser divergences (all Brent runs / emitted sites), printed-AF ('%.4f') and QUAL differences."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
import polymutt_amd as pm  # noqa: E402
from oracle_binding import Oracle  # noqa: E402

nfam = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
prec = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-4
ped = bench.nuclear_pedigree(pm, nfam, 2)
pl, dm, ref = pm.synth_block_host(ped, n, 11)
ora = Oracle(ped, pm.Params.defaults(precision=prec))
o, oc = ora.run(pl, dm, ref)
for num in (pm.NUM_PRODUCT, pm.NUM_EXACT, pm.NUM_POLY):
    eng = pm.Engine(ped, pm.Params.defaults(numerics=num, precision=prec), max_batch=n)
    e, ec = eng.run(pl, dm, ref)
    eng.close()
    called = o["status"] == 0
    div = np.abs(e["varfreq"] - o["varfreq"]) > 1e-6
    runs = int(sum(((o["n_cfg"] > k) & called).sum() for k in range(1, 7)))
    ndiv = int(sum((div[:, k] & (o["n_cfg"] > k) & called).sum() for k in range(1, 7)))
    em = o["emit"] != 0
    af_e = np.array(["%.4f" % x for x in e["af"][em]])
    af_o = np.array(["%.4f" % x for x in o["af"][em]])
    q_e = (e["poly_qual"][em] + 0.5).astype(int)
    q_o = (o["poly_qual"][em] + 0.5).astype(int)
    rel = np.max(np.abs(e["varllk"][called] - o["varllk"][called]) / np.maximum(np.abs(o["varllk"][called]), 1e-300))
    print(f"numerics={num} prec={prec}: brent runs {runs}, minimiser divergences {ndiv}; emitted {int(em.sum())}, "
          f"emitted with divergent AF {int((np.abs(e['af'][em]-o['af'][em])>1e-6).sum())}, printed-AF diffs "
          f"{int((af_e != af_o).sum())}, QUAL diffs {int((q_e != q_o).sum())}, maxidx diffs "
          f"{int((e['maxidx'] != o['maxidx']).sum())}, max llk rel err {rel:.2e}", flush=True)
