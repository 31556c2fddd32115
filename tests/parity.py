"""Engine-vs-oracle comparison with the tolerances of BASELINE.json's north star:
integer/byte/index fields bit-exact, likelihood/quality floats within 1e-6 (we hold much tighter)."""
import numpy as np

EXACT = ["status", "n_cfg", "maxidx", "emit", "total_depth", "num_samp_with_data", "allele1", "allele2",
         "is_mono", "denovo_mono", "call_row", "avg_map_qual", "perc_samp_with_data"]
LLK_RTOL = 1e-9      # log10-likelihoods: OCML log10 (<=1 ulp) + reduction order, ~1e-13 observed
FREQ_ATOL = 1e-6     # Brent minimiser / AF
QUAL_ATOL = 1e-6
FLAT_RTOL = 1e-12    # |llk_engine - llk_oracle| / |llk| at which an objective counts as flat
DOSE_ATOL = 1e-9


def compare_results(eng, ora, ecalls, ocalls, label="", dosage=True):
    """Returns a dict of mismatch counts; raises AssertionError with details on any failure.
    dosage=False: vcf_mode rows carry no dosage (FamilyLikelihoodSeq_VCF::OutputVCF prints none)."""
    assert len(eng) == len(ora)
    problems = []
    for f in EXACT:
        bad = np.nonzero(eng[f] != ora[f])[0]
        if len(bad):
            i = bad[0]
            problems.append(f"{label}{f}: {len(bad)} sites differ, first site {i}: engine {eng[f][i]} oracle {ora[f][i]}")
    called = ora["status"] == 0
    ncfg = ora["n_cfg"]
    flat_div = nonflat_div = runs = 0
    for k in range(7):
        m = called & (ncfg > k)
        if not m.any():
            continue
        e, o = eng["varllk"][m, k], ora["varllk"][m, k]
        rel = np.abs(e - o) / np.maximum(np.abs(o), 1e-300)
        if (rel > LLK_RTOL).any():
            i = np.argmax(rel)
            problems.append(f"{label}varllk[{k}] rel err {rel[i]:.3g} (engine {e[i]!r} oracle {o[i]!r})")
        if k > 0:
            # A Brent minimiser may differ where the objective is flat to rounding noise (e.g. a
            # configuration whose two alleles no read supports: every family term is the same constant
            # times (f+g)^4).  Such a divergence is recognised by the likelihoods at both minimisers
            # agreeing to FLAT_RTOL; any other divergence fails the comparison.
            d = np.abs(eng["varfreq"][m, k] - ora["varfreq"][m, k]) > FREQ_ATOL
            flat = rel <= FLAT_RTOL
            flat_div += int((d & flat).sum())
            nonflat_div += int((d & ~flat).sum())
            runs += int(m.sum())
    for f, tol in [("var_post_prob", 1e-9), ("poly_qual", QUAL_ATOL)]:
        d = np.abs(eng[f][called] - ora[f][called])
        if (d > tol).any():
            problems.append(f"{label}{f} max abs err {d.max():.3g}")
    if nonflat_div:
        problems.append(f"{label}{nonflat_div} minimiser divergences on non-flat objectives in {runs} Brent runs")
    em = ora["emit"] != 0
    for f, tol in [("af", FREQ_ATOL), ("ab", 1e-9), ("denovo_lr", QUAL_ATOL)]:
        d = np.abs(eng[f][em] - ora[f][em])
        if (d > tol).any():
            problems.append(f"{label}{f} max abs err {d.max():.3g} at site {np.nonzero(em)[0][np.argmax(d)]}")
    assert ecalls.shape == ocalls.shape, (ecalls.shape, ocalls.shape)
    for f in ["best", "gq", "label"]:
        bad = np.argwhere(ecalls[f] != ocalls[f])
        if len(bad):
            r, p = bad[0]
            problems.append(f"{label}calls.{f}: {len(bad)} differ; first row {r} person {p}: engine {ecalls[f][r, p]} oracle {ocalls[f][r, p]}")
    d = np.abs(ecalls["dosage"] - ocalls["dosage"]) if dosage else np.zeros(0)
    if d.size and (d > DOSE_ATOL).any():
        problems.append(f"{label}calls.dosage max abs err {d.max():.3g}")
    eval_mismatch = int(((eng["evals"] != ora["evals"]) & called[:, None]).any(axis=1).sum())
    assert not problems, "\n".join(problems)
    return {"sites": len(eng), "called": int(called.sum()), "emitted": int(em.sum()), "eval_path_mismatch": eval_mismatch,
            "flat_divergence": flat_div, "nonflat_divergence": nonflat_div, "brent_runs": runs}
