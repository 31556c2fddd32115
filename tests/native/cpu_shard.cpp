// tests/native/cpu_shard.cpp -- TEST HARNESS ONLY.
// libpm_cpu_driver.so: pmh_run_polymutt (include/polymutt_host.h) with the CPU oracle as the evaluator, so
// polymutt_amd/launch.py can run the product's sharded driver on CPU ranks (gloo) in the CPU test suite.
#include "../../include/polymutt_host.h"
#include "oracle_eval.h"

extern "C" int pmh_run_polymutt(int argc, char** argv, int32_t rank, int32_t world, int32_t device,
                                pmh_allgather_fn allgather, void* ctx) {
  (void)device;
  pmhost::ShardComm comm;
  comm.rank = rank;
  comm.world = world;
  if (world > 1 || allgather)
    comm.allgather = [=](const int64_t* send, int n, int64_t* recv) {
      if (allgather(ctx, send, n, recv) != 0) throw pmhost::FatalError("shard exchange (allgather) failed\n");
    };
  return pmhost::polymutt_main(argc, argv, &comm, oracle_factory());
}
