"""Static lane occupancy of the schedule compiler's generated ES functions (no device needed).

    python tools/es_occupancy.py [--shape ext10] [--families 200] [--seed 7] [--out profiles/r05_es_occupancy.json]

Writes the bench's synthetic pedigree of the shape (the same call bench.py makes), runs tests/native/build/jit_check
on it with PM_JIT_LAYOUT=1 and collects the compiler's `occupancy` lines: per generated wave-kernel function
(es_hoist_wave, --denovo engines: the bi-allelic / 10-state / top variants and the parts: leaf prefix, per-item
rest, top rest; the BA engines' thread-per-family es_hoist_jit has one lane per family and is not listed) the useful FP64 element-ops,
the lane slots its phases issue (a phase over E elements on WL lanes: ceil(E / WL) passes; a packed run of r type-2
steps: 10 r of WL lanes) and their ratio.  Functions of one shape repeat per chromosome class and engine kind; the
summary keeps each distinct (function, part, WL, ops, slots) once.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="ext10")
    ap.add_argument("--families", type=int, default=200)
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r05_es_occupancy.json"))
    a = ap.parse_args()
    import polymutt_amd as pm
    exe = os.path.join(ROOT, "tests", "native", "build", "jit_check")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "polymutt_amd"), "../tests/native/build/jit_check"], check=True)
    with tempfile.TemporaryDirectory() as d:
        pm.synth_write_dataset(d, a.shape, a.families, 1, a.seed)
        r = subprocess.run([exe, os.path.join(d, "test.dat"), os.path.join(d, "test.ped"), "--emit", os.path.join(d, "k.hip")],
                           capture_output=True, text=True, timeout=600, env=dict(os.environ, PM_JIT_LAYOUT="1"))
    if r.returncode != 0:
        sys.exit(r.stdout + r.stderr)
    seen, rows = set(), []
    for line in r.stderr.splitlines():
        if not line.startswith("occupancy"):
            continue
        # occupancy NAME part P WL W: OPS FP64 ops / SLOTS lane slots = OCC
        f = line.replace(":", "").split()
        key = (f[1], int(f[3]), int(f[5]), float(f[6]), float(f[10]))
        if key in seen:
            continue
        seen.add(key)
        rows.append({"function": f[1], "part": key[1], "lanes_per_family": key[2], "fp64_ops": key[3],
                     "lane_slots": key[4], "occupancy": float(f[-1])})
    kinds = {}
    for row in rows:
        kind = row["function"].split("_", 1)[1] if "_" in row["function"] else row["function"]
        kind = {"0": "biallelic", "1": "10state", "2": "top"}.get(kind, kind)
        k = kinds.setdefault(kind, {"ops": 0.0, "slots": 0.0, "min": 1.0, "max": 0.0})
        k["ops"] += row["fp64_ops"]; k["slots"] += row["lane_slots"]
        k["min"] = min(k["min"], row["occupancy"]); k["max"] = max(k["max"], row["occupancy"])
    summary = {kind: {"occupancy": v["ops"] / v["slots"] if v["slots"] else 0.0, "min": v["min"], "max": v["max"]}
               for kind, v in sorted(kinds.items())}
    out = {"shape": a.shape, "families": a.families, "seed": a.seed,
           "source": "tests/native/build/jit_check with PM_JIT_LAYOUT=1 (csrc/es_jit.cpp gen_wave_family / gen_family)",
           "by_kind": summary, "functions": rows}
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    for kind, v in summary.items():
        print(f"{kind:10s} occupancy {v['occupancy']:.3f} (functions {v['min']:.3f}-{v['max']:.3f})")


if __name__ == "__main__":
    main()
