#!/usr/bin/env python3
"""Generate the reference-pinned golden fixtures under tests/golden/synth/.

TEST INFRASTRUCTURE.  Runs only in the build container, where /root/reference exists and
oracle/_ref/pm_ref (the reference's own objects linked by oracle/ref/ref_harness.cpp) can be built.
For every case below it

  1. writes a synthetic GLF dataset with the product's generator (SURVEY.md 8(d) recipe),
  2. runs the reference harness on it (--dump_sites: per-site varllk[7]/varfreq[7]/evals/...,
     --out_vcf: the VCF the reference CLI would write),
  3. stores the per-site dump as plain arrays (.npz, no pickles), the VCF body (non-## lines, gzip)
     and the SHA-256 of the dense input block, so tests can regenerate the inputs and prove they are
     the ones the reference saw.

Usage: python tools/make_golden.py [case ...]
"""
import gzip
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tests", "golden", "synth")
PM_REF = os.path.join(ROOT, "oracle", "_ref", "pm_ref")

# name: (shape, families, sites, seed, extra CLI flags[, extras]); extras: {"pos": [[label, position], ...]} writes the
# --pos file pos.txt; "cli_only": the case is checked through the CLI's VCF only (several sections or --pos)
CASES = {
    "quad_auto": ("quad", 30, 400, 7, []),
    "trio_auto": ("trio", 30, 400, 11, []),
    "mixed_auto": ("mixed", 31, 400, 5, []),
    "single_auto": ("single", 20, 300, 3, []),
    "single_one_nuclear": ("quad", 1, 400, 13, []),
    "ext10_auto": ("ext10", 10, 300, 17, []),
    "roof_auto": ("roof", 12, 300, 19, []),
    "quad_denovo": ("quad+dn", 30, 400, 7, ["--denovo", "--rate_denovo", "1e-6"]),
    "trio_denovo": ("trio+dn", 30, 400, 23, ["--denovo", "--rate_denovo", "1e-5"]),
    "ext10_denovo": ("ext10+dn", 10, 300, 29, ["--denovo", "--rate_denovo", "1e-6"]),
    "mixed_denovo": ("mixed+dn", 31, 300, 71, ["--denovo", "--rate_denovo", "1e-5"]),
    "quad_denovo_plain": ("quad", 30, 300, 73, ["--denovo"]),
    "quad_chrX": ("quad", 30, 400, 31, ["--chrX", "1"]),
    "quad_chrY": ("quad", 30, 400, 37, ["--chrY", "1"]),
    "quad_MT": ("quad", 30, 400, 41, ["--MT", "1"]),
    "mixed_chrX": ("mixed", 31, 400, 43, ["--chrX", "1"]),
    "ext10_chrX": ("ext10", 10, 300, 47, ["--chrX", "1"]),
    "quad_quick": ("quad", 30, 400, 53, ["--quick_call"]),
    "quad_filters": ("quad", 30, 400, 59, ["--minDepth", "2150", "--maxDepth", "2300", "-c", "0.9",
                                           "--minPercSampleWithData", "99.5"]),
    "quad_allsites": ("quad", 10, 300, 61, ["--all_sites"]),
    "quad_prec": ("quad", 30, 400, 67, ["--prec", "1e-6", "--theta", "0.01", "--poly_tstv", "1.5"]),
    # ES type-3 peels (parents -> only child) under the 10-state de novo model and on chrX
    "roof_denovo": ("roof+dn", 12, 300, 83, ["--denovo", "--rate_denovo", "1e-6"]),
    "roof_chrX": ("roof", 12, 300, 89, ["--chrX", "1"]),
    # type-3 peel WITH a marriage partial (a roof created by UpdateRoof): BA, --denovo (:1391), chrX
    "roof2_auto": ("roof2", 10, 300, 103, []),
    "roof2_denovo": ("roof2+dn", 10, 300, 107, ["--denovo", "--rate_denovo", "1e-6"]),
    "roof2_chrX": ("roof2", 10, 300, 109, ["--chrX", "1"]),
    # BASELINE.json config geometries (the lane plans and kernels the bench selects for them)
    "big_trio_1000": ("trio", 1000, 256, 11, []),
    "big_quad_1000_denovo": ("quad", 1000, 256, 7, ["--denovo"]),
    "big_ext10_200": ("ext10", 200, 256, 17, []),
    "big_ext10_200_denovo": ("ext10+dn", 200, 256, 29, ["--denovo", "--rate_denovo", "1e-6"]),
    # config 4 at its stated 8-12-member range: ext10, roof, roof2, ext12 (6 founders), ext11 (5 founders) dealt
    # round-robin, so every launch mixes schedules and polynomial degrees D = 8, 10, 12
    "extmix_auto": ("extmix", 15, 300, 151, []),
    "extmix_denovo": ("extmix+dn", 10, 300, 157, ["--denovo", "--rate_denovo", "1e-6"]),
    "extmix_chrX": ("extmix", 15, 300, 163, ["--chrX", "1"]),
    "big_extmix_200": ("extmix", 200, 256, 167, []),
    "big_extmix_200_denovo": ("extmix+dn", 200, 256, 173, ["--denovo", "--rate_denovo", "1e-6"]),
    # a few extended pedigrees next to > 512 nuclear families
    "big_quadext_600": ("quadext", 600, 256, 97, []),
    "big_quadext_600_denovo": ("quadext", 600, 200, 101, ["--denovo", "--rate_denovo", "1e-6"]),
    # CLI surface of the site loop (main.cpp:286-308, :332-337, :593; OutputVCF's PL columns :1751-1830)
    "quad_gl_off": ("quad", 20, 300, 113, ["--gl_off"]),
    "quad_pos": ("quad", 20, 300, 127, ["--pos", "pos.txt"],
                 {"pos": [["1", p] for p in range(5, 301, 13)], "cli_only": True}),
    "quad_pos_missing": ("quad", 20, 300, 139, ["--pos", "pos.txt"],
                         {"pos": [["1", p] for p in range(3, 301, 29)] + [["1", 5000], ["2", 7]], "cli_only": True}),
    "multi_all": ("quad+multi", 20, 200, 131, [], {"cli_only": True}),
    "multi_chr2process": ("trio+multi", 20, 200, 137, ["--chr2process", "2,X"], {"cli_only": True}),
    "multi_chr2process_one": ("quad+multi", 20, 200, 149, ["--chr2process", "2"], {"cli_only": True}),
}

SITE_DUMP = np.dtype([("pos", "<i4"), ("ref", "<i4"), ("status", "<i4"), ("total_depth", "<i4"),
                      ("num_samp_with_data", "<i4"), ("avg_map_qual", "<f8"), ("perc_samp_with_data", "<f8"),
                      ("n_cfg", "<i4"), ("maxidx", "<i4"), ("var_post_prob", "<f8"), ("poly_qual", "<f8"),
                      ("varllk", "<f8", (7,)), ("varfreq", "<f8", (7,)), ("evals", "<i4", (7,)),
                      ("emitted", "<i4"), ("denovo_lr", "<f8")])
assert SITE_DUMP.itemsize == 212


def block_sha256(directory):
    """SHA-256 over (ref, pl, dm) of every section as the product GLF reader decodes them."""
    import polymutt_amd as pm
    ped = pm.Pedigree(os.path.join(directory, "test.dat"), os.path.join(directory, "test.ped"))
    cwd = os.getcwd()
    os.chdir(directory)
    try:
        rd = pm.GlfReader(ped, "test.gif")
        h = hashlib.sha256()
        for label, maxpos in rd.sections():   # synthetic sections: one record per position
            pos, ref, pl, dm = rd.read(maxpos + 16)
            for a in (pos, ref, pl, dm):
                h.update(np.ascontiguousarray(a).tobytes())
        return h.hexdigest()
    finally:
        os.chdir(cwd)


def make_case(name):
    import polymutt_amd as pm
    shape, nfam, nsites, seed, flags = CASES[name][:5]
    extras = CASES[name][5] if len(CASES[name]) > 5 else {}
    tmp = tempfile.mkdtemp(prefix="pm_gold_")
    try:
        pm.synth_write_dataset(tmp, shape, nfam, nsites, seed)
        if "pos" in extras:
            with open(os.path.join(tmp, "pos.txt"), "w") as fh:
                fh.write("".join(f"{l} {p}\n" for l, p in extras["pos"]))
        cmd = [PM_REF, "-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--out_vcf", "out.vcf",
               "--dump_sites", "sites.bin"] + flags
        r = subprocess.run(cmd, cwd=tmp, capture_output=True, text=True, timeout=600)
        if r.returncode != 0:
            raise RuntimeError(f"{name}: reference harness failed:\n{r.stdout[-2000:]}")
        dump = np.fromfile(os.path.join(tmp, "sites.bin"), dtype=SITE_DUMP)
        arrays = {f: dump[f] for f in SITE_DUMP.names}
        np.savez_compressed(os.path.join(OUT, name + ".npz"), **arrays)
        body = [l for l in open(os.path.join(tmp, "out.vcf")).read().splitlines() if not l.startswith("##")] \
            if os.path.exists(os.path.join(tmp, "out.vcf")) else []
        with gzip.GzipFile(os.path.join(OUT, name + ".vcf.gz"), "wb", mtime=0) as fh:
            fh.write(("\n".join(body) + "\n").encode() if body else b"")
        summary = [l for l in r.stdout.splitlines() if l.strip() and not l.startswith("Analysis")
                   and "started" not in l and "ended" not in l and "Time" not in l]
        out = {"shape": shape, "families": nfam, "sites": nsites, "seed": seed, "flags": flags,
               "block_sha256": block_sha256(tmp), "records": max(0, len(body) - 1), "dumped_sites": int(len(dump))}
        out.update(extras)
        if extras.get("cli_only"):   # the summary block the reference printed (wall-clock lines dropped)
            out["summary"] = [l for l in r.stdout.splitlines() if l.startswith(("Summary of", "Total ", "Non-Poly", "Transi",
                              "Transv", "Other ", "Filter", "\t", "Hard ", "Skipped"))]
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def main():
    if not os.path.exists(PM_REF):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "ref"], check=True)
    os.makedirs(OUT, exist_ok=True)
    names = sys.argv[1:] or list(CASES)
    meta_path = os.path.join(OUT, "cases.json")
    meta = json.load(open(meta_path)) if os.path.exists(meta_path) else {}
    for n in names:
        meta[n] = make_case(n)
        print(n, meta[n]["dumped_sites"], "sites,", meta[n]["records"], "records", flush=True)
        with open(meta_path, "w") as fh:
            json.dump(meta, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
