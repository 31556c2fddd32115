#!/usr/bin/env python3
"""tools/cpu_calibrate.py -- TEST/MEASUREMENT INFRASTRUCTURE (build container only).

Calibrates the clean-room CPU restatement (tests/native/build/cpu_polymutt: the product host driver with the
serial oracle oracle/pm_oracle.c as evaluator) against the reference itself (oracle/_ref/pm_ref, built from
/root/reference by oracle/ref/Makefile) on identical synthetic GLF inputs, so that bench.py's cpu_baseline
(which times the restatement on the GPU box's host cores: the reference's objects never travel there,
license.txt:1) can state how it relates to the reference.  Two slice sizes per run give the steady-state
per-site rate with start-up (pedigree load, 4000 GLF opens) subtracted: rate = (S2 - S1) / (t2 - t1).

    python tools/cpu_calibrate.py [--families 1000] [--sites 200 2000] [--threads 1 4 8] > profiles/r03_cpu_calibration.json
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
    ap.add_argument("--sites", type=int, nargs=2, default=[200, 2000])
    ap.add_argument("--threads", type=int, nargs="+", default=[1, 4, 8])
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
    for name, exe, threads in [("port", port, [1])] + [("reference", ref, a.threads)]:
        for t in threads:
            t1, b1 = run(exe, dirs[s1], t, a.denovo)
            t2, b2 = run(exe, dirs[s2], t, a.denovo)
            out["runs"][f"{name}_{t}"] = {"seconds": [t1, t2], "steady_sites_per_s": (s2 - s1) / (t2 - t1),
                                          "end_to_end_sites_per_s": s2 / t2, "vcf_body": b2}
    body = out["runs"]["port_1"].pop("vcf_body")
    for k, v in out["runs"].items():
        v["vcf_identical_to_port"] = v.pop("vcf_body", body) == body
    port_rate = out["runs"]["port_1"]["steady_sites_per_s"]
    best = max((v["steady_sites_per_s"], k) for k, v in out["runs"].items() if k.startswith("reference"))
    out["reference_1thread_over_port"] = out["runs"]["reference_1"]["steady_sites_per_s"] / port_rate
    out["reference_best_over_port"] = best[0] / port_rate
    out["reference_best_threads"] = best[1]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
