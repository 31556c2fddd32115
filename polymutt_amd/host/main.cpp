// main.cpp -- the `polymutt` command line (src/main.cpp:57-627 surface) on the MI355X engine.
// The site loop body runs on the GPU through the C ABI (include/polymutt_engine.h); there is no CPU
// fallback: without a usable HIP device the program exits with an error.  Multi-GPU runs go through
// polymutt_amd/launch.py (one process per GPU, pmh_run_polymutt).
#include "../../include/polymutt_host.h"

int main(int argc, char** argv) { return pmh_run_polymutt(argc, argv, 0, 1, -1, nullptr, nullptr); }
