// main.cpp -- the `polymutt` command line (src/main.cpp:57-627 surface) on the MI355X engine.
// The site loop body runs on the GPU through the C ABI (include/polymutt_engine.h); there is no CPU
// fallback: without a usable HIP device the program exits with an error.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../../include/polymutt_engine.h"
#include "blocks.h"
#include "driver.h"

using namespace pmhost;

class EngineEvaluator : public SiteEvaluator {
 public:
  EngineEvaluator(const pm_pedigree& ped, const pm_params& par, int device, int batch) {
    int rc = pm_engine_create(&ped, &par, device, batch, &eng_);
    if (rc) throw FatalError(std::string("GPU engine initialisation failed: ") + pm_last_error() + "\n");
  }
  ~EngineEvaluator() { pm_engine_destroy(eng_); }
  void begin_section(int chrom) override { check(pm_engine_begin_section(eng_, chrom)); }
  void run(int n, const uint8_t* pl, const uint32_t* dm, const uint8_t* ref, pm_site_result* res, pm_geno_call* calls,
           int* n_rows) override {
    int rc = pm_engine_run(eng_, n, pl, dm, ref, 0, res, calls, n_rows);
    if (rc == PM_EBRENT) { printf("\nFATAL NUMERIC ERROR - ScalarMinimizer::Brent got stuck\n\n"); exit(1); }
    check(rc);
  }
  void counters(pm_counters* out) override { check(pm_engine_counters(eng_, out)); }

 private:
  static void check(int rc) { if (rc) throw FatalError(std::string("GPU engine error: ") + pm_last_error() + "\n"); }
  pm_engine* eng_ = nullptr;
};

int main(int argc, char** argv) {
  try {
    Options opt = parse_command_line(argc, argv);
    Pedigree ped;
    ped.load(opt.datFile, opt.pedFile);
    if (!opt.blocksOut.empty()) {   // --glf2blocks: GLF site stream -> dense indexed blocks, no engine
      if (opt.glfListFile.empty()) throw FatalError("--glf2blocks needs the GLF index file (-g)\n");
      const long n = convert_glf_to_blocks(ped, opt.glfListFile, opt.blocksOut, default_io_threads(opt), opt.blockSites);
      printf("%ld sites written to %s\n", n, opt.blocksOut.c_str());
      return 0;
    }
    pm_pedigree v = ped.view();
    pm_params par = opt.params();
    const auto t0 = std::chrono::steady_clock::now();
    EngineEvaluator ev(v, par, opt.device, opt.batch);
    if (getenv("PM_TIMING"))
      fprintf(stderr, "PM_TIMING engine create %.3f s\n",
              std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    return run_polymutt(opt, ped, ev);
  } catch (const FatalError& e) {
    printf("\nFATAL ERROR - \n%s\n\n", e.what());
    return 1;
  }
}
