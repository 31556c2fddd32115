"""An --in_vcf input with the record kinds example/testvcf.in.vcf lacks (it holds only biallelic SNVs):
multi-allelic and REF == ALT records, which the reference drops (src/FamilyLikelihoodSeq_VCF.cpp:296-301,
OutputVCF :419), indels, which it calls with alleles 1/2 (:303-306), and a lower-case ALT (Allele2Int
:65-72).  Built by editing the committed example input, so the untouched records keep their golden lines."""
import gzip
import os

from conftest import EXAMPLE

# record index -> (REF, ALT) replacement
EDITS = {
    10: (None, "T,G"),    # multi-allelic: not output
    20: (None, "C"),      # REF == ALT: not output
    30: ("CA", None),     # deletion: indel, alleles 1/2
    40: (None, "AT"),     # insertion: indel, alleles 1/2
    50: (None, "t"),      # lower-case SNV allele
    700: (None, "A,C,G"),
    701: ("C", "C"),
    702: ("CTT", "C"),
}
DROPPED = {10, 20, 700, 701}
INDELS = {30, 40, 702}


def write_edited_vcf(path):
    """Writes the edited input (plain text) and returns the number of records."""
    lines = gzip.open(os.path.join(EXAMPLE, "testvcf.in.vcf.gz"), "rt").read().splitlines()
    out, k = [], 0
    for l in lines:
        if l.startswith("#"):
            out.append(l)
            continue
        if k in EDITS:
            c = l.split("\t")
            ref, alt = EDITS[k]
            if ref is not None:
                c[3] = ref
            if alt is not None:
                c[4] = alt
            l = "\t".join(c)
        out.append(l)
        k += 1
    with open(path, "w") as fh:
        fh.write("\n".join(out) + "\n")
    return k


def golden_records():
    return gzip.open(os.path.join(EXAMPLE, "testvcf.out.vcf.body.gz"), "rt").read().splitlines()[1:]


def check_edited_output(got, theta=0.001, n_founders=6):
    """The output records for the edited input against the reference's golden for the original input:
    dropped records absent; untouched records byte-identical; the lower-case SNV identical but for its ALT
    column; an indel identical but for REF/ALT and QUAL, where QUAL moves by the prior term the indel branch
    uses (PedVCF.cpp:136-152: log10(prior) instead of the precedence-slipped log10(p_ts or p_tv))."""
    import math
    gold = golden_records()
    n = len(gold)
    kept = [i for i in range(n) if i not in DROPPED]
    assert len(got) == len(kept), (len(got), len(kept))
    prior = theta * sum(1.0 / i for i in range(1, 2 * n_founders + 1))
    ts = {("A", "G"), ("G", "A"), ("C", "T"), ("T", "C")}
    for j, i in enumerate(kept):
        g, e = got[j].split("\t"), gold[i].split("\t")
        if i in INDELS:
            assert g[:3] == e[:3] and g[6:] == e[6:], i
            ref, alt = EDITS[i]
            assert (g[3], g[4]) == (ref or e[3], alt or e[4]), i
            p_snv = 2.0 / 3.0 if (e[3], e[4]) in ts else 1.0 / 6.0
            q_gold = float(e[5])
            if q_gold > 100.0:   # both QUALs are 10 x the log-likelihood difference (no posterior clamp)
                assert abs(float(g[5]) - (q_gold + 10 * (math.log10(prior) - math.log10(p_snv)))) <= 0.011, (i, g[5], e[5])
        elif i in EDITS:
            assert g[:4] == e[:4] and g[4] == EDITS[i][1] and g[5:] == e[5:], i
        else:
            assert got[j] == gold[i], f"record {i} differs:\n{got[j][:200]}\n{gold[i][:200]}"


def _zero_pl(col):
    """A sample column with its PL replaced by 0,0,0 (no data: withdata_cnt counts a sample only when one of
    its three values is non-zero, FamilyLikelihoodSeq_VCF.cpp:345-350)."""
    f = col.split(":")
    f[-1] = "0,0,0"
    return ":".join(f)


def _drop_dp(cols):
    """The record with its DP FORMAT key renamed (GT:GQ:DP:DS:PL -> GT:GQ:XD:DS:PL): DP is then absent, while PL
    keeps the FORMAT index the first biallelic record fixes for the whole file (:316-324)."""
    fmt = cols[8].split(":")
    fmt[fmt.index("DP")] = "XD"
    return cols[:8] + [":".join(fmt)] + cols[9:]


def write_nodata_vcf(path, worlds=(2, 3), empty_rank=None):
    """The example input edited so that the records a shard rank meets first carry no data (all PL 0,0,0): the
    reference prints them with the previous computed record's QUAL, AF and genotypes (PedVCF.cpp:113-122), so a
    sharded run must hand that state over from the rank before.  The first line of every rank's byte slice
    (polymutt_amd/host/vcf_input.cpp) for each world size is blanked with its neighbours; the first three records
    have no DP key (DP's FORMAT index is looked up per record until found, :316-324); empty_rank=(r, world)
    blanks that rank's whole slice (the state then comes from two ranks back).  Returns the blanked record indices."""
    lines = gzip.open(os.path.join(EXAMPLE, "testvcf.in.vcf.gz"), "rt").read().splitlines()
    head = [l for l in lines if l.startswith("#")]
    recs = [l.split("\t") for l in lines if not l.startswith("#")]
    for i in range(3):
        recs[i] = _drop_dp(recs[i])

    def layout():
        body = sum(len(l) + 1 for l in head)
        starts, off = [], body
        for r in recs:
            starts.append(off)
            off += len("\t".join(r)) + 1
        return body, off, starts

    blank = set()
    body, total, starts = layout()   # blanking changes lengths: the slices are taken on the final file below
    for _ in range(3):               # fixed point: blank, recompute the slices, blank again
        for w in worlds:
            for r in range(1, w):
                lo = body + (total - body) * r // w
                k = next(i for i, s in enumerate(starts) if s >= lo)
                blank.update(range(max(0, k - 2), min(len(recs), k + 3)))
        if empty_rank:
            r, w = empty_rank
            lo, hi = body + (total - body) * r // w, body + (total - body) * (r + 1) // w
            blank.update(i for i, s in enumerate(starts) if lo <= s < hi)
        for i in blank:
            recs[i] = recs[i][:9] + [_zero_pl(c) for c in recs[i][9:]]
        body, total, starts = layout()
    for w in worlds:   # every rank's first record is blanked in the final layout
        for r in range(1, w):
            lo = body + (total - body) * r // w
            assert next(i for i, s in enumerate(starts) if s >= lo) in blank, (w, r)
    with open(path, "w") as fh:
        fh.write("\n".join(head + ["\t".join(r) for r in recs]) + "\n")
    return sorted(blank)
