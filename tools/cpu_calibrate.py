#!/usr/bin/env python3
"""tools/cpu_calibrate.py -- TEST/MEASUREMENT INFRASTRUCTURE (build container only).

Calibrates the clean-room CPU restatement (tests/native/build/cpu_polymutt: the product host driver with the
oracle oracle/pm_oracle.c as evaluator, built with the reference's OpenMP sections) against the reference itself (oracle/_ref/pm_ref, built from
/root/reference by oracle/ref/Makefile) on identical synthetic GLF inputs, so that bench.py's cpu_baseline
(which times the restatement on the GPU box's host cores: the reference's objects never travel there,
license.txt:1) can state how it relates to the reference.  Two slice sizes per run give the steady-state
per-site rate with start-up (pedigree load, 4000 GLF opens) subtracted: rate = (S2 - S1) / (t2 - t1).  Both
programs run at every thread count (default 1 and 4: the 8-CPU build container is oversubscribed at 8), best of
--reps runs, and the ratio reference / restatement is reported per thread count.

    python tools/cpu_calibrate.py [--families 1000] [--sites 200 1000] [--threads 1 4] > profiles/r04_cpu_calibration.json
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(exe, d, threads, denovo):
    cmd = [exe, "-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--out_vcf", "o.vcf", "--nthreads", str(threads)]
    cmd += ["--denovo"] if denovo else []
    t0 = time.perf_counter()
    r = subprocess.run(cmd, cwd=d, capture_output=True, text=True, env=dict(os.environ, OMP_NUM_THREADS=str(threads)))
    dt = time.perf_counter() - t0
    if r.returncode:
        sys.exit(f"{exe} failed: {r.stdout[-400:]}")
    body = [l for l in open(os.path.join(d, "o.vcf")).read().splitlines() if not l.startswith("##")]
    return dt, body


def main():
    import polymutt_amd as pm
    ap = argparse.ArgumentParser()
    ap.add_argument("--families", type=int, default=1000)
    ap.add_argument("--shape", default="quad")
    ap.add_argument("--sites", type=int, nargs=2, default=[200, 1000])
    ap.add_argument("--threads", type=int, nargs="+", default=[1, 4])
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--no-denovo", dest="denovo", action="store_false", default=True)
    a = ap.parse_args()
    port = os.path.join(ROOT, "tests", "native", "build", "cpu_polymutt")
    ref = os.path.join(ROOT, "oracle", "_ref", "pm_ref")
    tmp = tempfile.mkdtemp(prefix="pm_cal_")
    dirs = {}
    for s in a.sites:
        dirs[s] = os.path.join(tmp, str(s))
        pm.synth_write_dataset(dirs[s], a.shape, a.families, s, 7)
    out = {"workload": f"{a.families} {a.shape} families, seed 7" + (", --denovo" if a.denovo else ""),
           "slices": a.sites, "nproc": os.cpu_count(), "runs": {}}
    s1, s2 = a.sites
    for name, exe in [("port", port), ("reference", ref)]:
        for t in a.threads:
            best = None
            for _ in range(a.reps):
                t1, b1 = run(exe, dirs[s1], t, a.denovo)
                t2, b2 = run(exe, dirs[s2], t, a.denovo)
                best = (t1, t2, b2) if best is None else (min(best[0], t1), min(best[1], t2), b2)
            t1, t2, b2 = best
            out["runs"][f"{name}_{t}"] = {"seconds": [t1, t2], "steady_sites_per_s": (s2 - s1) / (t2 - t1),
                                          "end_to_end_sites_per_s": s2 / t2, "vcf_body": b2}
    body = out["runs"]["port_1"]["vcf_body"]
    for k, v in out["runs"].items():
        v["vcf_identical_to_port"] = v.pop("vcf_body") == body
    out["reference_over_port"] = {str(t): out["runs"][f"reference_{t}"]["steady_sites_per_s"] /
                                  out["runs"][f"port_{t}"]["steady_sites_per_s"] for t in a.threads}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
