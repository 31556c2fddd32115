#!/usr/bin/env python3
"""Generate the reference-pinned GLF-ingest fixture under tests/golden/ingest/.

TEST INFRASTRUCTURE.  Runs only in the build container, where oracle/_ref/pm_ref (the reference's own
objects, built by oracle/ref/Makefile from /root/reference) exists.

The dense synthetic fixtures give every person a record at every position.  This one exercises the
PedigreeGLF merge (src/PedigreeGLF.cpp:197-324) on ragged input, which is what the parallel ingest
(polymutt_amd/host/ingest.cpp) restates:
  * persons with different position sets (a site is the minimum position over the open files; persons
    without a record there are absent from it),
  * the refBase of a site taken from the first person holding the minimum, with refBase disagreements,
  * indel records (type 2, skipped by NextBaseEntry) and records at the same position as the previous one
    (offset 0), which repeat a site,
  * a person whose section ends early (its end record ends the section for everybody),
  * a person without a GLF key in the index (a null handle: absent everywhere), and two sections.

Writes test.ped/test.dat/test.gif, the GLF files (gzip), and the VCF body the reference writes for them.
Usage: python tools/make_ingest_golden.py
"""
import gzip
import os
import random
import shutil
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "tests", "golden", "ingest")
PM_REF = os.path.join(ROOT, "oracle", "_ref", "pm_ref")
NFAM, MAXPOS = 6, 400
BASES = [1, 2, 4, 8]   # IUPAC bitmasks of A, C, G, T (glfHandler translateBase)
GENO = [(a, b) for a in range(4) for b in range(a, 4)]   # AA AC AG AT CC CG CT GG GT TT


def record(rng, off, ref_mask, alt):
    """A type-1 record: a genotype close to (ref, alt) gets PL 0, the others grow with distance."""
    ref = BASES.index(ref_mask) if ref_mask in BASES else 0
    truth = rng.choice([(ref, ref), (ref, alt), (alt, alt)])
    lk = []
    for g in GENO:
        d = (g[0] != truth[0]) + (g[1] != truth[1]) + (g[0] != truth[1]) + (g[1] != truth[0])
        lk.append(0 if g == tuple(sorted(truth)) else min(255, 10 * d + rng.randrange(0, 40)))
    depth, mapq = rng.randrange(1, 30), rng.choice([20, 37, 60])
    return struct.pack("<BIIB10B", (1 << 4) | ref_mask, off, depth | (0 << 24), mapq, *lk)


def indel(rng, off):
    l0, l1 = rng.randrange(1, 4), -rng.randrange(1, 3)
    seq = bytes(rng.choice(b"ACGT") for _ in range(abs(l0))) + bytes(rng.choice(b"ACGT") for _ in range(abs(l1)))
    return struct.pack("<BIIB3Bhh", (2 << 4) | 1, off, 9, 60, 0, 30, 60, l0, l1) + seq


def person_glf(rng, person, early_end):
    out = bytearray(b"GLF\x03") + struct.pack("<I", 0)
    for sec, label in enumerate([b"1", b"2"]):
        out += struct.pack("<i", len(label) + 1) + label + b"\x00" + struct.pack("<i", MAXPOS)
        last = 0
        top = 150 if (early_end and sec == 0) else 300
        for p in range(1, top + 1):
            if rng.random() < 0.15:   # this person has no record here
                continue
            if rng.random() < 0.03:   # an indel record at this position, skipped by NextBaseEntry
                out += indel(rng, p - last)
                last = p
            ref_mask = BASES[(p * 7 + sec) % 4] if rng.random() > 0.05 else BASES[(p * 7 + sec + 1) % 4]
            alt = ((p * 7 + sec) % 4 + 2) % 4
            out += record(rng, p - last, ref_mask, alt)
            last = p
            if rng.random() < 0.01:   # a second record at the same position (offset 0)
                out += record(rng, 0, ref_mask, alt)
        out += b"\x00"   # end-of-section record (recordType 0)
    return bytes(out)


def main():
    if not os.path.exists(PM_REF):
        sys.exit("oracle/_ref/pm_ref is missing: build it with `make -C oracle ref` (needs /root/reference)")
    rng = random.Random(2027)
    shutil.rmtree(OUT, ignore_errors=True)
    os.makedirs(OUT)
    ped, gif = [], []
    n = 0
    for f in range(NFAM):
        for k in range(4):
            n += 1
            fa, mo = (0, 0) if k < 2 else (n - k + 0, n - k + 1)
            ped.append(f"F{f}\t{n}\t{fa}\t{mo}\t{1 + k % 2}\t{n}")
            if n != 11:   # person 11 has no GLF key in the index: a null handle
                gif.append(f"{n} p{n}.glf.gz")
    open(os.path.join(OUT, "test.ped"), "w").write("\n".join(ped) + "\n")
    open(os.path.join(OUT, "test.dat"), "w").write("T\tGLF_Index\n")
    open(os.path.join(OUT, "test.gif"), "w").write("\n".join(gif) + "\n")
    for p in range(1, n + 1):
        if p == 11:
            continue
        with gzip.open(os.path.join(OUT, f"p{p}.glf.gz"), "wb", compresslevel=9) as fh:
            fh.write(person_glf(rng, p, early_end=(p == 17)))
    with tempfile.TemporaryDirectory() as tmp:
        vcf = os.path.join(tmp, "out.vcf")
        r = subprocess.run([PM_REF, "-p", "test.ped", "-d", "test.dat", "-g", "test.gif", "--out_vcf", vcf, "--all_sites"],
                           cwd=OUT, capture_output=True, text=True)
        if r.returncode != 0:
            sys.exit(r.stdout[-2000:] + r.stderr[-2000:])
        body = [l for l in open(vcf).read().splitlines() if not l.startswith("##")]
    with gzip.open(os.path.join(OUT, "ref.vcf.body.gz"), "wt") as fh:
        fh.write("\n".join(body) + "\n")
    print(f"{len(body) - 1} records -> {OUT}")


if __name__ == "__main__":
    main()
