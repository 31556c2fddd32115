#!/usr/bin/env python3
"""Summarise a tools/profile_round.sh run (gpurun_out/prof_ROUND) into committed files under profiles/:

  profiles/ROUND_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary of the default bench command
  profiles/ROUND_kernel_stats_1engine.csv   ... of the same workload on one engine (kernels never overlap)
  profiles/ROUND_kernel_stats_ext10.csv     ... of BASELINE config 4's shape (200 ext10 pedigrees), one engine
  profiles/ROUND_bench*.json        the bench JSON lines printed under those profiler runs
  profiles/ROUND_pmc.json           per kernel (one-engine bench): dispatches and mean FETCH_SIZE / WRITE_SIZE /
                                    SQ counters per dispatch, plus HBM bytes per dispatch with the gfx950 correction
                                    (MI355X_MICROARCH.md "HBM": FETCH_SIZE counts 1/2 of the bytes -> x2)
  profiles/ROUND_fp64_peak.json     measured FP64 issue rates (tools/fp64_peak.hip)
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    n = name.split("(")[0].replace("void ", "")
    return n


def pmc_summary(src, subs):
    """Per kernel: dispatches and mean counters per dispatch over the PMC pass directories `subs`."""
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    src_of = {}   # counter -> the pass it was collected in
    for sub in subs:
        path = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(path):
            continue
        for row in csv.DictReader(open(path)):
            k = short(row["Kernel_Name"])
            acc[k][row["Counter_Name"]] += float(row["Counter_Value"])
            disp[(k, sub)].add(row["Dispatch_Id"])
            src_of[row["Counter_Name"]] = sub
    out = {}
    for k, counters in acc.items():
        d = {}
        for c, v in counters.items():
            sub = src_of[c]
            n = max(1, len(disp[(k, sub)]))
            d[c + "_per_dispatch"] = v / n
            d["dispatches_" + sub] = n
        if "SQ_WAVE_CYCLES_per_dispatch" in d:
            for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                if c + "_per_dispatch" in d:
                    d[c + "_frac_of_wave_cycles"] = d[c + "_per_dispatch"] / d["SQ_WAVE_CYCLES_per_dispatch"]
        if "FETCH_SIZE_per_dispatch" in d:
            # FETCH_SIZE / WRITE_SIZE are reported in KiB
            d["hbm_read_bytes_per_dispatch"] = 2 * d["FETCH_SIZE_per_dispatch"] * 1024
        if "WRITE_SIZE_per_dispatch" in d:
            d["hbm_write_bytes_per_dispatch"] = d["WRITE_SIZE_per_dispatch"] * 1024
        out[k] = d
    return out


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{rnd}")
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    for sub, suffix in (("trace", "_3engines"), ("trace1", "_1engine"), ("trace_ext10", "_ext10"), ("trace_ext10dn", "_ext10dn"),
                        ("trace_cfg5", "_cfg5"), ("trace_extmix", "_extmix")):
        if not os.path.exists(os.path.join(src, sub, "run_kernel_stats.csv")):
            continue
        shutil.copy(os.path.join(src, sub, "run_kernel_stats.csv"), os.path.join(dst, f"{rnd}_kernel_stats{suffix}.csv"))
        bench = [l for l in open(os.path.join(src, sub + ".out")).read().splitlines() if l.startswith("{")]
        if bench:
            with open(os.path.join(dst, f"{rnd}_bench{suffix}.json"), "w") as fh:
                fh.write(bench[-1] + "\n")
    if os.path.exists(os.path.join(src, "bench.out")):   # the default bench line (3 engines, cpu_baseline)
        bench = [l for l in open(os.path.join(src, "bench.out")).read().splitlines() if l.startswith("{")]
        if bench:
            with open(os.path.join(dst, f"{rnd}_bench.json"), "w") as fh:
                fh.write(bench[-1] + "\n")
    others = []
    for name in ("cfg2", "cfg3plain", "cfg4", "cfg4dn", "cfg4mix", "cfg4mixdn", "cfg5"):
        path = os.path.join(src, name + ".out")
        if os.path.exists(path):
            lines = [l for l in open(path).read().splitlines() if l.startswith("{")]
            if lines:
                d = json.loads(lines[-1])
                d["profile_step"] = name
                others.append(json.dumps(d))
    if others:
        with open(os.path.join(dst, f"{rnd}_bench_other_configs.jsonl"), "w") as fh:
            fh.write("\n".join(others) + "\n")
    peak = [l for l in open(os.path.join(src, "fp64_peak.out")).read().splitlines() if l.startswith("{")]
    if peak:
        with open(os.path.join(dst, f"{rnd}_fp64_peak.json"), "w") as fh:
            fh.write(peak[-1] + "\n")
    out = pmc_summary(src, ("pmc_fetch", "pmc_write", "pmc_sq", "pmc_sq2", "pmc_sq3"))
    # the tree the passes ran on (profile_round.sh writes revision.txt from REVISION): bench.py stamps
    # roofline.traffic_source with it
    rev = "unknown"
    for cand in (os.path.join(src, "revision.txt"), os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "REVISION")):
        if os.path.exists(cand):
            rev = open(cand).read().split()[-1] if "revision:" in open(cand).read() else open(cand).read().strip()
            break
    out["revision"] = rev
    with open(os.path.join(dst, f"{rnd}_pmc.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)
    for tag, subs in (("ext10", ("pmc_ext10_fetch", "pmc_ext10_sq", "pmc_ext10_sq2")),   # config 4 BA: the fused kernel
                      ("ext10dn", ("pmc_ext10dn_sq", "pmc_ext10dn_sq2", "pmc_ext10dn_sq3")),   # --denovo: es_hoist_wave
                      ("cfg5", ("pmc_cfg5_fetch", "pmc_cfg5_sq", "pmc_cfg5_sq2"))):   # config 5
        e = pmc_summary(src, subs)
        if e:
            e["revision"] = rev
            with open(os.path.join(dst, f"{rnd}_pmc_{tag}.json"), "w") as fh:
                json.dump(e, fh, indent=1, sort_keys=True)
    print(json.dumps({k: ({kk: round(vv, 1) for kk, vv in v.items()} if isinstance(v, dict) else v) for k, v in out.items()}, indent=1))


if __name__ == "__main__":
    main()
