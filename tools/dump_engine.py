"""Run the engine (and optionally the oracle) over a GLF dataset and save per-site results (debug tool)."""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import polymutt_amd as pm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--dir", required=True)
ap.add_argument("--ped", default="test.ped")
ap.add_argument("--out", required=True)
ap.add_argument("--batch", type=int, default=4096)
ap.add_argument("--param", action="append", default=[])
a = ap.parse_args()
kw = {}
for p in a.param:
    k, v = p.split("=")
    kw[k] = float(v) if "." in v or "e" in v else int(v)
ped = pm.Pedigree(os.path.join(a.dir, "test.dat"), os.path.join(a.dir, a.ped))
cwd = os.getcwd()
os.chdir(a.dir)
rd = pm.GlfReader(ped, "test.gif")
os.chdir(cwd)
eng = pm.Engine(ped.view, pm.Params.defaults(**kw), max_batch=a.batch)
allres, allcalls = [], []
for lab, _ in rd.sections():
    eng.begin_section(0)
    while True:
        pos, ref, pl, dm = rd.read(a.batch)
        if len(pos) == 0:
            break
        r, c = eng.run(pl, dm, ref)
        allres.append(r)
        allcalls.append(c)
np.savez_compressed(a.out, res=np.concatenate(allres), calls=np.concatenate(allcalls))
print("saved", a.out)
