"""Reference-pinned synthetic fixtures (tests/golden/synth, written by tools/make_golden.py from the
reference's own objects): dataset regeneration, CLI-flag -> pm_params translation and the
per-site comparison against the reference's --dump_sites records."""
import gzip
import hashlib
import json
import os

import numpy as np

import polymutt_amd as pm

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SYNTH = os.path.join(ROOT, "tests", "golden", "synth")
CASES = json.load(open(os.path.join(SYNTH, "cases.json")))
# cases with one section and no --pos: also compared site by site against the reference's --dump_sites records
DUMP_CASES = sorted(n for n, c in CASES.items() if not c.get("cli_only"))
# cases the serial CPU oracle needs minutes for (10-state peels of 200 pedigrees): the oracle is pinned on the same
# shapes by their small cases (extmix_denovo), and the GPU engine is compared with these cases' reference dumps and
# VCFs directly, without an oracle run
ORACLE_SLOW = {"big_extmix_200_denovo"}


def summary_block(stdout):
    """The section-summary lines a run prints (main.cpp:596-619), as make_golden.py keeps them."""
    return [l for l in stdout.splitlines() if l.startswith(("Summary of", "Total ", "Non-Poly", "Transi", "Transv",
                                                             "Other ", "Filter", "\t", "Hard ", "Skipped"))]

LLK_RTOL = 1e-9
FREQ_ATOL = 1e-6
FLAT_RTOL = 1e-12


def make_dataset(name, directory):
    c = CASES[name]
    pm.synth_write_dataset(directory, c["shape"], c["families"], c["sites"], c["seed"])
    if "pos" in c:   # the --pos file the reference read
        with open(os.path.join(directory, "pos.txt"), "w") as fh:
            fh.write("".join(f"{l} {p}\n" for l, p in c["pos"]))
    return c


def read_dataset(directory):
    """Pedigree + every section's dense block, as the product GLF reader decodes them."""
    ped = pm.Pedigree(os.path.join(directory, "test.dat"), os.path.join(directory, "test.ped"))
    cwd = os.getcwd()
    os.chdir(directory)
    try:
        rd = pm.GlfReader(ped, "test.gif")
        secs = []
        h = hashlib.sha256()
        for label, maxpos in rd.sections():   # synthetic sections: one record per position
            pos, ref, pl, dm = rd.read(maxpos + 16)
            for a in (pos, ref, pl, dm):
                h.update(np.ascontiguousarray(a).tobytes())
            secs.append((label, pos, ref, pl, dm))
    finally:
        os.chdir(cwd)
    return ped, secs, h.hexdigest()


_FLAG_PARAMS = {"--theta": ("theta", float), "--poly_tstv": ("poly_tstv", float), "--prec": ("precision", float),
                "-c": ("posterior", float), "--minDepth": ("min_total_depth", int),
                "--maxDepth": ("max_total_depth", int), "--minPercSampleWithData": ("min_ps", float),
                "--minMapQuality": ("min_map_quality", int), "--rate_denovo": ("denovo_mut_rate", float),
                "--tstv_denovo": ("denovo_tstv", float), "--minLLR_denovo": ("denovo_min_llr", float)}
_FLAG_BOOL = {"--denovo": "denovo", "--all_sites": "all_sites", "--quick_call": "quick_call", "--gl_off": None}


def params_and_chrom(flags, **extra):
    """(pm_params, chromosome class of section "1") for a fixture's reference command line."""
    kw, chrom, i = {}, pm.PM_CHR_AUTO, 0
    while i < len(flags):
        f = flags[i]
        if f in _FLAG_BOOL:
            if _FLAG_BOOL[f]:   # (--gl_off only changes the VCF text)
                kw[_FLAG_BOOL[f]] = 1
            i += 1
            continue
        v = flags[i + 1]
        if f in _FLAG_PARAMS:
            k, t = _FLAG_PARAMS[f]
            kw[k] = t(v)
        elif f == "--chrX" and v == "1":
            chrom = pm.PM_CHR_X
        elif f == "--chrY" and v == "1":
            chrom = pm.PM_CHR_Y
        elif f == "--MT" and v == "1":
            chrom = pm.PM_CHR_MT
        else:
            raise ValueError(f"unhandled fixture flag {f}")
        i += 2
    kw.update(extra)
    return pm.Params.defaults(**kw), chrom


def golden_dump(name):
    with np.load(os.path.join(SYNTH, name + ".npz")) as z:
        return {k: z[k] for k in z.files}


def golden_vcf_body(name):
    return gzip.open(os.path.join(SYNTH, name + ".vcf.gz"), "rt").read().splitlines()


def compare_to_dump(res, dump, label=""):
    """Per-site results (pm_site_result array) against the reference harness's --dump_sites records.
    Integer fields exact; log10-likelihoods to LLK_RTOL; minimisers to FREQ_ATOL except where the
    objective is flat to rounding (then the likelihoods must still agree); emission exact."""
    problems = []
    n = len(dump["status"])
    assert len(res) == n, (len(res), n)
    st = dump["status"]
    if (res["status"] != st).any():
        i = int(np.nonzero(res["status"] != st)[0][0])
        problems.append(f"{label}status differs at {int((res['status'] != st).sum())} sites, first {i}: "
                        f"{res['status'][i]} vs reference {st[i]}")
    called = st == 0
    for f in ("total_depth", "num_samp_with_data"):
        m = st != 5
        if (res[f][m] != dump[f][m]).any():
            problems.append(f"{label}{f} differs")
    for f in ("avg_map_qual", "perc_samp_with_data"):
        m = st != 5
        if (res[f][m] != dump[f][m]).any():
            problems.append(f"{label}{f} differs")
    for f in ("n_cfg", "maxidx"):
        if (res[f][called] != dump[f][called]).any():
            i = int(np.nonzero((res[f] != dump[f]) & called)[0][0])
            problems.append(f"{label}{f} differs at site {i}: {res[f][i]} vs reference {dump[f][i]}")
    flat = nonflat = runs = 0
    for k in range(7):
        m = called & (dump["n_cfg"] > k)
        if not m.any():
            continue
        e, o = res["varllk"][m, k], dump["varllk"][m, k]
        rel = np.abs(e - o) / np.maximum(np.abs(o), 1e-300)
        if (rel > LLK_RTOL).any():
            i = int(np.argmax(rel))
            problems.append(f"{label}varllk[{k}] rel err {rel[i]:.3g} ({e[i]!r} vs reference {o[i]!r})")
        if k > 0:   # see tests/parity.py: divergences on flat objectives are allowed, no others
            d = np.abs(res["varfreq"][m, k] - dump["varfreq"][m, k]) > FREQ_ATOL
            flat += int((d & (rel <= FLAT_RTOL)).sum())
            nonflat += int((d & (rel > FLAT_RTOL)).sum())
            runs += int(m.sum())
    if nonflat:
        problems.append(f"{label}{nonflat} minimiser divergences on non-flat objectives in {runs} Brent runs")
    d = np.abs(res["var_post_prob"][called] - dump["var_post_prob"][called])
    if d.size and d.max() > 1e-9:
        problems.append(f"{label}var_post_prob max abs err {d.max():.3g}")
    d = np.abs(res["poly_qual"][called] - dump["poly_qual"][called])
    if d.size and d.max() > 1e-6:
        problems.append(f"{label}poly_qual max abs err {d.max():.3g}")
    # the harness flags every site that reaches OutputVCF(_denovo); emit==2 is a de novo record that
    # OutputVCF_denovo itself suppresses (denovoLR < minLLR)
    emitted = (res["emit"] != 0).astype(np.int32)
    if (emitted != dump["emitted"]).any():
        i = int(np.nonzero(emitted != dump["emitted"])[0][0])
        problems.append(f"{label}emitted differs at {int((emitted != dump['emitted']).sum())} sites, first {i}")
    em = dump["emitted"] == 1
    d = np.abs(res["denovo_lr"][em] - dump["denovo_lr"][em])
    if d.size and d.max() > 1e-6 * max(1.0, np.abs(dump["denovo_lr"][em]).max()):
        problems.append(f"{label}denovo_lr max abs err {d.max():.3g}")
    # The harness counts calls of the virtual Brent objective f(); the engine and oracle also count the
    # direct likelihood evaluations that bypass it (de novo mono, the lone-nuclear-family eval at 0.5),
    # so a reference count of 0 matches 0 or 1.
    ev, dv = res["evals"], dump["evals"]
    diff = (ev != dv) & ~((dv == 0) & (ev == 1))
    eval_path = int((diff & called[:, None]).any(axis=1).sum())
    assert not problems, "\n".join(problems)
    return {"sites": n, "called": int(called.sum()), "emitted": int(em.sum()), "flat_divergence": flat,
            "nonflat_divergence": nonflat, "brent_runs": runs, "eval_path_mismatch": eval_path}
