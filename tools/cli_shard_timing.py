#!/usr/bin/env python3
"""tools/cli_shard_timing.py -- end-to-end timing of the drop-in CLI on dense indexed blocks (--in_blocks) with one
process and with N processes on the same GPU (polymutt_amd/launch.py; each rank seeks to its own blocks, so no rank
reads another's, polymutt_amd/host/blocks.cpp), plus a byte comparison of the two VCFs.  Prints one JSON line.

    python tools/cli_shard_timing.py [--families 1000] [--sites 20000] [--ranks 2] [--denovo]
"""
import argparse
import json
import os
import re
import shutil
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def body(path):
    return [l for l in open(path).read().splitlines() if not l.startswith("##")]


def main():
    import polymutt_amd as pm
    ap = argparse.ArgumentParser()
    ap.add_argument("--families", type=int, default=1000)
    ap.add_argument("--sites", type=int, default=20000)
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--denovo", action="store_true")
    a = ap.parse_args()
    tmp = tempfile.mkdtemp(prefix="pm_shard_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        t0 = time.perf_counter()
        pm.synth_write_dataset(tmp, "quad", a.families, a.sites, 7)
        t_synth = time.perf_counter() - t0
        base = [pm.BIN_PATH, "-p", "test.ped", "-d", "test.dat"]
        extra = ["--denovo"] if a.denovo else []
        t0 = time.perf_counter()
        r = subprocess.run(base + ["-g", "test.gif", "--glf2blocks", "in.pmb"], cwd=tmp, capture_output=True, text=True, timeout=900)
        t_convert = time.perf_counter() - t0
        assert r.returncode == 0, r.stdout[-2000:]
        env = dict(os.environ, PM_BLOCK_STATS="1")
        t0 = time.perf_counter()
        r1 = subprocess.run(base + ["--in_blocks", "in.pmb", "--out_vcf", "one.vcf"] + extra, cwd=tmp, capture_output=True,
                            text=True, timeout=900, env=env)
        t_one = time.perf_counter() - t0
        assert r1.returncode == 0, r1.stdout[-2000:]
        env2 = dict(env, PYTHONPATH=ROOT + os.pathsep + env.get("PYTHONPATH", ""), OMP_NUM_THREADS="1")

        def launch(cwd, pmb, out):
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                port = s.getsockname()[1]
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(a.ranks),
                   "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "polymutt_amd.launch"] + base[1:] + \
                  ["--in_blocks", pmb, "--out_vcf", out] + extra
            t0 = time.perf_counter()
            r = subprocess.run(cmd, cwd=cwd, capture_output=True, text=True, timeout=900, env=env2)
            assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
            return time.perf_counter() - t0, r

        # start-up of the multi-process run (torchrun, torch import, process group, engines) on a 64-site input
        small = os.path.join(tmp, "small")
        pm.synth_write_dataset(small, "quad", a.families, 64, 7)
        r = subprocess.run(base + ["-g", "test.gif", "--glf2blocks", "small.pmb"], cwd=small, capture_output=True, text=True, timeout=900)
        assert r.returncode == 0, r.stdout[-2000:]
        t_overhead, _ = launch(small, "small.pmb", "small.vcf")
        t0 = time.perf_counter()
        r1s = subprocess.run(base + ["--in_blocks", "small.pmb", "--out_vcf", "s1.vcf"] + extra, cwd=small, capture_output=True,
                             text=True, timeout=900)
        t_overhead1 = time.perf_counter() - t0
        t_shard, r2 = launch(tmp, "in.pmb", "sharded.vcf")
        blocks = {}
        for m in re.finditer(r"PM_BLOCK_STATS shard (\d+) section (\S+): blocks read (\d+)", r2.stderr):
            blocks[int(m.group(1))] = blocks.get(int(m.group(1)), 0) + int(m.group(3))
        same = body(os.path.join(tmp, "one.vcf")) == body(os.path.join(tmp, "sharded.vcf"))
        print(json.dumps({"families": a.families, "sites": a.sites, "denovo": a.denovo, "ranks": a.ranks,
                          "gpus": "one (all ranks share it; gloo exchange)", "pmb_bytes": os.path.getsize(os.path.join(tmp, "in.pmb")),
                          "seconds_synth_glf": t_synth, "seconds_glf2blocks": t_convert, "seconds_1_process": t_one,
                          f"seconds_{a.ranks}_processes": t_shard, "sites_per_s_1_process": a.sites / t_one,
                          f"sites_per_s_{a.ranks}_processes": a.sites / t_shard,
                          "startup_seconds_1_process": t_overhead1, f"startup_seconds_{a.ranks}_processes": t_overhead,
                          "sites_per_s_1_process_past_startup": a.sites / max(1e-9, t_one - t_overhead1),
                          f"sites_per_s_{a.ranks}_processes_past_startup": a.sites / max(1e-9, t_shard - t_overhead),
                          "blocks_read_per_rank": blocks,
                          "vcf_identical": same, "records": len(body(os.path.join(tmp, "one.vcf"))) - 1}), flush=True)
        return 0 if same else 1
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == "__main__":
    sys.exit(main())
