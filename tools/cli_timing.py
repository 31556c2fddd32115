#!/usr/bin/env python3
"""tools/cli_timing.py -- end-to-end timing of the drop-in `polymutt` CLI on one GPU (measurement tooling).

  --in_blocks: 1000 synthetic quads x --sites sites written as GLF, converted once with --glf2blocks, then the CLI on
  the .pmb for each --engines / --batch setting.  Start-up (pedigree load, engine creation, file opens) is measured
  on a 64-site input and subtracted; PM_TIMING=1 gives each pipeline stage's busy seconds (ingest thread, engine
  stage, VCF writer).  Every setting's VCF body must equal the first one's.
  --in_vcf: a synthetic VCF of the BASELINE config-5 shape (2000 mixed trio/quad families, GT:PL per sample, the
  engine's own site generator for the PLs) through `polymutt --in_vcf`.

Prints one JSON object (profiles/r04_cli_*.json).

    python tools/cli_timing.py [--sites 100000] [--engines 1 2 3] [--batch 4096 16384] [--vcf-records 20000]
"""
import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def body(path):
    with open(path) as fh:
        return [l for l in fh if not l.startswith("##")]


def timing_fields(stderr):
    out = {}
    m = re.search(r"PM_TIMING ingest ([\d.]+) s, engine ([\d.]+) s, vcf ([\d.]+) s", stderr)
    if m:
        out = {"ingest_busy_s": float(m.group(1)), "engine_stage_busy_s": float(m.group(2)), "vcf_busy_s": float(m.group(3))}
    m = re.search(r"PM_TIMING vcf input: read ([\d.]+) s, classify ([\d.]+) s, parse ([\d.]+) s, engine ([\d.]+) s, "
                  r"format ([\d.]+) s, write ([\d.]+) s", stderr)
    if m:
        for k, v in zip(("read", "classify", "parse", "engine", "format", "write"), m.groups()):
            out["vcf_" + k + "_s"] = float(v)
    m = re.search(r"PM_TIMING open inputs ([\d.]+) s", stderr)
    if m:
        out["open_inputs_s"] = float(m.group(1))
    m = re.search(r"PM_TIMING wall: first batch ([\d.]+) s, ingest done ([\d.]+) s, end ([\d.]+) s", stderr)
    if m:
        out.update({"wall_first_batch_s": float(m.group(1)), "wall_ingest_done_s": float(m.group(2)), "wall_end_s": float(m.group(3))})
    m = re.search(r"PM_TIMING first window: section ([\d.]+) s, sites ([\d.]+) s, fill ([\d.]+) s", stderr)
    if m:
        out.update({"wall_section_s": float(m.group(1)), "wall_first_sites_s": float(m.group(2)), "wall_first_fill_s": float(m.group(3))})
    m = re.search(r"PM_TIMING glf ingest: .*decode ahead ([\d.]+) s", stderr)
    if m:
        out["glf_decode_ahead_s"] = float(m.group(1))
    m = re.search(r"PM_TIMING engine create ([\d.]+) s", stderr)
    if m:
        out["engine_create_s"] = float(m.group(1))
    return out


def run_cli(args, cwd, timeout=1200, extra_env=None):
    env = dict(os.environ, PM_TIMING="1", **(extra_env or {}))
    t0 = time.perf_counter()
    r = subprocess.run(args, cwd=cwd, capture_output=True, text=True, timeout=timeout, env=env)
    dt = time.perf_counter() - t0
    if r.returncode != 0:
        raise SystemExit(f"{' '.join(args)} failed:\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}")
    return dt, r


def write_vcf(pm, d, families, records, seed):
    """A VCF for --in_vcf of the config-5 shape: the .ped of `families` mixed families (synth_write_dataset) and, per
    record, REF = the site's reference base, ALT = its transition, PL of every sample from the engine's synthetic
    generator's three planes of (REF, ALT)."""
    pm.synth_write_dataset(d, "mixed", families, 1, seed)
    ped = pm.Pedigree(os.path.join(d, "test.dat"), os.path.join(d, "test.ped"))
    pids = ped.pids()
    np_ = ped.n_person
    bases = "NACGT"
    ts = [0, 3, 4, 1, 2]

    def gi(a, b):
        a, b = min(a, b), max(a, b)
        return (a - 1) * (10 - a) // 2 + (b - a)
    with open(os.path.join(d, "in.vcf"), "w") as fh:
        fh.write("##fileformat=VCFv4.1\n##FORMAT=<ID=GT,Number=1,Type=String,Description=\"Genotype\">\n"
                 "##FORMAT=<ID=PL,Number=3,Type=Integer,Description=\"Phred-scaled Genotype Likelihoods\">\n")
        fh.write("#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT\t" + "\t".join(pids) + "\n")
        chunk = 2048
        distinct = []   # the first 2048 records are generated; later ones repeat them at new positions (speed)
        for s0 in range(0, records, chunk):
            n = min(chunk, records - s0)
            if distinct:
                fh.write("".join(f"1\t{s0 + i + 1}\t{distinct[i % len(distinct)]}" for i in range(n)))
                continue
            pl, dm, ref = pm.synth_block_host(ped.view, n, seed, s0)
            pl = pl.reshape(n, np_, 10)
            lines = []
            for i in range(n):
                r = int(ref[i]) if 1 <= int(ref[i]) <= 4 else 1
                a = ts[r]
                trip = pl[i][:, [gi(r, r), gi(r, a), gi(a, a)]]
                strs = np.char.add(np.char.add(np.char.add("0/1:", trip[:, 0].astype(str)), ","),
                                   np.char.add(np.char.add(trip[:, 1].astype(str), ","), trip[:, 2].astype(str)))
                lines.append(f"1\t{s0 + i + 1}\t.\t{bases[r]}\t{bases[a]}\t50\tPASS\t.\tGT:PL\t" + "\t".join(strs.tolist()))
            fh.write("\n".join(lines) + "\n")
            distinct = [l.split("\t", 2)[2] + "\n" for l in lines]
    return np_


def main():
    import polymutt_amd as pm
    ap = argparse.ArgumentParser()
    ap.add_argument("--families", type=int, default=1000)
    ap.add_argument("--sites", type=int, default=100000)
    ap.add_argument("--engines", type=int, nargs="+", default=[1, 2, 3])
    ap.add_argument("--batch", type=int, nargs="+", default=[4096, 16384])
    ap.add_argument("--denovo", action="store_true")
    ap.add_argument("--vcf-records", type=int, default=0, help="also time --in_vcf on a config-5 VCF of this many records")
    ap.add_argument("--vcf-families", type=int, default=2000)
    ap.add_argument("--keep", default=None, help="work directory to keep (default: a temporary one, removed)")
    ap.add_argument("--glf", action="store_true", help="also time the CLI on the GLF files themselves (the reference's input)")
    ap.add_argument("--vcf-only", action="store_true", help="only the --in_vcf timing (no GLF / block runs)")
    ap.add_argument("--no-blocks", action="store_true", help="skip the --in_blocks runs (with --glf: GLF runs only)")
    ap.add_argument("--glf-env", nargs="+", default=[""], help="GLF runs under each of these env settings (K=V,K2=V2)")
    ap.add_argument("--vcf-small", type=int, default=2000, help="--in_vcf start-up run: records (subtracted for the steady rate)")
    a = ap.parse_args()
    tmp = a.keep or tempfile.mkdtemp(prefix="pm_cli_", dir=os.environ.get("TMPDIR", "/tmp"))
    os.makedirs(tmp, exist_ok=True)
    out = {"families": a.families, "sites": a.sites, "denovo": a.denovo, "runs": []}
    try:
        base = [pm.BIN_PATH, "-p", "test.ped", "-d", "test.dat"]
        extra = ["--denovo"] if a.denovo else []
        if not a.vcf_only:
            t0 = time.perf_counter()
            pm.synth_write_dataset(tmp, "quad", a.families, a.sites, 7)
            out["seconds_synth_glf"] = time.perf_counter() - t0
            if not a.no_blocks:
                out["seconds_glf2blocks"], _ = run_cli(base + ["-g", "test.gif", "--glf2blocks", "in.pmb"], tmp)
                out["pmb_bytes"] = os.path.getsize(os.path.join(tmp, "in.pmb"))
            small = os.path.join(tmp, "small")
            pm.synth_write_dataset(small, "quad", a.families, 64, 7)
            if not a.no_blocks:
                run_cli(base + ["-g", "test.gif", "--glf2blocks", "small.pmb"], small)
            ref_body = None
            for e in ([] if a.no_blocks else a.engines):
                for b in a.batch:
                    # start-up (a 64-site run) and the full run, each the best of 3: single start-up samples varied
                    # 0.48-0.85 s on one box, which made their difference meaningless
                    t_small = min(run_cli(base + ["--in_blocks", "small.pmb", "--out_vcf", "s.vcf", "--engines", str(e), "--batch", str(b)] + extra,
                                          small)[0] for _ in range(3))
                    runs = [run_cli(base + ["--in_blocks", "in.pmb", "--out_vcf", "o.vcf", "--engines", str(e), "--batch", str(b)] + extra, tmp)
                            for _ in range(3)]
                    dt, r = min(runs, key=lambda x: x[0])
                    bd = body(os.path.join(tmp, "o.vcf"))
                    if ref_body is None:
                        ref_body = bd
                    rec = {"engines": e, "batch": b, "seconds": dt, "startup_seconds": t_small, "sites_per_s": a.sites / dt,
                           "sites_per_s_past_startup": a.sites / max(1e-9, dt - t_small), "records": len(bd) - 1,
                           "vcf_identical_to_first": bd == ref_body}
                    rec.update(timing_fields(r.stderr))
                    out["runs"].append(rec)
                    print(json.dumps(rec), file=sys.stderr, flush=True)
            if a.glf:   # the drop-in on GLF: decode, merge and fill in the ingest thread; start-up from the 64-site GLF set
                for e, genv in [(e, g) for e in a.engines for g in a.glf_env]:
                    xe = dict(kv.split("=", 1) for kv in genv.split(",") if kv)
                    # (best of 5: the 64-site start-up runs varied 1.28-1.65 s between calls on one box)
                    small_best = min((run_cli(base + ["-g", "test.gif", "--out_vcf", "s.vcf", "--engines", str(e)] + extra, small,
                                              extra_env=xe) for _ in range(5)), key=lambda x: x[0])
                    t_small = small_best[0]
                    runs = [run_cli(base + ["-g", "test.gif", "--out_vcf", "g.vcf", "--engines", str(e)] + extra, tmp, extra_env=xe)
                            for _ in range(5)]
                    dt, r = min(runs, key=lambda x: x[0])
                    bd = body(os.path.join(tmp, "g.vcf"))
                    rec = {"input": "glf", "env": genv, "engines": e, "seconds": dt, "startup_seconds": t_small, "sites_per_s": a.sites / dt,
                           "sites_per_s_past_startup": a.sites / max(1e-9, dt - t_small), "records": len(bd) - 1,
                           "vcf_identical_to_blocks": ref_body is None or bd == ref_body}
                    rec.update(timing_fields(r.stderr))
                    rec["small_timing"] = timing_fields(small_best[1].stderr)
                    if "wall_end_s" in rec:   # in the pipeline: the sites after the first batch over the wall time after it
                        rec["sites_per_s_pipeline"] = (a.sites - 4096) / max(1e-9, rec["wall_end_s"] - rec["wall_first_batch_s"])
                    m = re.search(r"PM_TIMING glf ingest: decode ([\d.]+) s, merge ([\d.]+) s, fill ([\d.]+) s", r.stderr)
                    if m:
                        rec.update({"glf_decode_s": float(m.group(1)), "glf_merge_s": float(m.group(2)), "glf_fill_s": float(m.group(3))})
                    out.setdefault("glf_runs", []).append(rec)
                    print(json.dumps(rec), file=sys.stderr, flush=True)
                out["glf_best"] = max(out["glf_runs"], key=lambda x: x["sites_per_s_past_startup"])
            if out["runs"]:
                best = max(out["runs"], key=lambda x: x["sites_per_s_past_startup"])
                out["best"] = {k: best[k] for k in ("engines", "batch", "sites_per_s", "sites_per_s_past_startup")}
            out["all_vcf_identical"] = all(x["vcf_identical_to_first"] for x in out["runs"])
        if a.vcf_records:
            vd = os.path.join(tmp, "vcf")
            os.makedirs(vd, exist_ok=True)
            t0 = time.perf_counter()
            npers = write_vcf(pm, vd, a.vcf_families, a.vcf_records, 11)
            t_write = time.perf_counter() - t0
            vbytes = os.path.getsize(os.path.join(vd, "in.vcf"))
            big = min((run_cli(base + ["--in_vcf", "in.vcf", "--out_vcf", "o.vcf"], vd) for _ in range(3)), key=lambda x: x[0])
            t_one = big[0]
            # the steady rate: a small VCF of the same samples (the first records of in.vcf) timed the same way, subtracted
            with open(os.path.join(vd, "in.vcf")) as fi, open(os.path.join(vd, "small.vcf"), "w") as fo:
                n = 0
                for l in fi:
                    if not l.startswith("#"):
                        n += 1
                        if n > a.vcf_small:
                            break
                    fo.write(l)
            small_r = min((run_cli(base + ["--in_vcf", "small.vcf", "--out_vcf", "s.vcf"], vd) for _ in range(3)), key=lambda x: x[0])
            t_small = small_r[0]
            out["in_vcf"] = {"families": a.vcf_families, "samples": npers, "records": a.vcf_records, "vcf_bytes": vbytes,
                             "seconds_write": t_write, "seconds": t_one, "records_per_s": a.vcf_records / t_one,
                             "small_records": a.vcf_small, "small_seconds": t_small,
                             "records_per_s_steady": (a.vcf_records - a.vcf_small) / max(1e-9, t_one - t_small),
                             "MB_per_s": vbytes / t_one / 1e6, "records_out": len(body(os.path.join(vd, "o.vcf"))) - 1,
                             "timing": timing_fields(big[1].stderr), "small_timing": timing_fields(small_r[1].stderr)}
        print(json.dumps(out, indent=1), flush=True)
        return 0 if out.get("all_vcf_identical", True) else 1
    finally:
        if not a.keep:
            shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    sys.exit(main())
