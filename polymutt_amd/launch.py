"""Multi-GPU `polymutt`: one process per GPU, each analysing a contiguous position range of every section
(sites shard with no data-path exchange).

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m polymutt_amd.launch -p test.ped -d test.dat -g test.gif --out_vcf out.vcf [polymutt flags]

Rank r runs the product driver (pmh_run_polymutt, include/polymutt_host.h) on GPU LOCAL_RANK.  At each
section end the ranks exchange one small int64 vector (the section counters of src/main.cpp:264-282, the
entry count, how many sites reached OutputVCF, the byte range of the shard's records) with one all-gather:
summing the gathered counters is the single counter all-reduce, and the rest orders the VCF merge.  Rank 0
prints the summed section summaries (main.cpp:596-619) and concatenates the shards' records behind the
header; the result is byte-identical to a one-process run (tests/test_cpu_host.py, tests/test_gpu_engine.py).

Collective backend: RCCL ("nccl") when every local rank has its own GPU, else gloo (CPU tests, or several
ranks sharing one GPU).  --lib selects another build of pmh_run_polymutt (the CPU tests pass the oracle one).

PM_COLLECTIVE=nccl|gloo forces the backend, and at WORLD_SIZE 1 (still under torchrun) runs the sharded protocol
over one rank -- the per-section all-gather then runs on the one GPU's RCCL communicator, so the exchange path of a
multi-GPU run is exercised on a one-GPU box (tests/test_gpu_engine.py::test_cli_rccl_exchange_world_one).
"""
import ctypes as C
import os
import sys

import numpy as np

_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_int64), C.c_int32, C.POINTER(C.c_int64))


def run(argv, lib_path=None):
    import torch
    import torch.distributed as dist
    from . import engine

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    lib = C.CDLL(lib_path or engine.LIB_PATH)
    lib.pmh_run_polymutt.restype = C.c_int
    lib.pmh_run_polymutt.argtypes = [C.c_int, C.POINTER(C.c_char_p), C.c_int32, C.c_int32, C.c_int32, _FN, C.c_void_p]
    args = ["polymutt"] + list(argv)
    cargv = (C.c_char_p * len(args))(*[a.encode() for a in args])
    forced = os.environ.get("PM_COLLECTIVE", "")
    if forced not in ("", "nccl", "gloo"):
        print(f"PM_COLLECTIVE={forced}: expected nccl or gloo", file=sys.stderr)
        return 2
    if world <= 1 and not forced:
        return lib.pmh_run_polymutt(len(args), cargv, 0, 1, -1, _FN(0), None)

    ngpu = torch.cuda.device_count()   # counts devices without initialising HIP in this process
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    use_rccl = (forced == "nccl") if forced else (lib_path is None and ngpu >= local_world)
    if use_rccl and ngpu == 0:
        print("PM_COLLECTIVE=nccl needs a GPU", file=sys.stderr)
        return 2
    device = local % ngpu if ngpu > 0 else -1
    if use_rccl:
        torch.cuda.set_device(device)
    dist.init_process_group("nccl" if use_rccl else "gloo")
    dev = torch.device("cuda", device) if use_rccl else torch.device("cpu")

    if rank == 0 and forced:
        print(f"polymutt_amd.launch: collective backend {dist.get_backend()}, world {world}", file=sys.stderr)

    def allgather(_ctx, send, n, recv):
        try:
            t = torch.from_numpy(np.ctypeslib.as_array(send, shape=(n,)).copy()).to(dev)
            out = torch.empty(world * n, dtype=torch.int64, device=dev)
            dist.all_gather_into_tensor(out, t)
            np.ctypeslib.as_array(recv, shape=(world * n,))[:] = out.cpu().numpy()
            return 0
        except Exception as e:   # the driver turns a failed exchange into its FATAL ERROR exit
            print(f"rank {rank}: allgather failed: {e}", file=sys.stderr)
            return 1

    cb = _FN(allgather)
    if rank > 0:   # the reference's stdout (banner, section summaries) comes from rank 0 only
        sys.stdout.flush()
        devnull = os.open(os.devnull, os.O_WRONLY)
        os.dup2(devnull, 1)
    try:
        rc = lib.pmh_run_polymutt(len(args), cargv, rank, world, device if lib_path is None else -1, cb, None)
    finally:
        dist.destroy_process_group()
    return rc


def main():
    argv = sys.argv[1:]
    lib_path = None
    if len(argv) >= 2 and argv[0] == "--lib":
        lib_path, argv = argv[1], argv[2:]
    sys.exit(run(argv, lib_path))


if __name__ == "__main__":
    main()
