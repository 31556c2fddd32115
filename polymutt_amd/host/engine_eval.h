// engine_eval.h -- the HIP engine behind the driver's SiteEvaluator boundary (the product evaluator).
// There is no CPU fallback: without a usable HIP device pm_engine_create fails and the run stops.
#pragma once
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include "../../include/polymutt_engine.h"
#include "driver.h"

namespace pmhost {

class EngineEvaluator : public SiteEvaluator {
 public:
  EngineEvaluator(const pm_pedigree& ped, const pm_params& par, int device, int batch) {
    const auto t0 = std::chrono::steady_clock::now();
    int rc = pm_engine_create(&ped, &par, device, batch, &eng_);
    if (rc) throw FatalError(std::string("GPU engine initialisation failed: ") + pm_last_error() + "\n");
    if (getenv("PM_TIMING"))
      fprintf(stderr, "PM_TIMING engine create %.3f s\n", std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  }
  ~EngineEvaluator() override { pm_engine_destroy(eng_); }
  void begin_section(int chrom) override { check(pm_engine_begin_section(eng_, chrom)); }
  void run(int n, const uint8_t* pl, const uint32_t* dm, const uint8_t* ref, pm_site_result* res, pm_geno_call* calls,
           int* n_rows) override {
    int rc = pm_engine_run(eng_, n, pl, dm, ref, 0, res, calls, n_rows);
    if (rc == PM_EBRENT) { printf("\nFATAL NUMERIC ERROR - ScalarMinimizer::Brent got stuck\n\n"); exit(1); }
    check(rc);
  }
  void counters(pm_counters* out) override { check(pm_engine_counters(eng_, out)); }
  void set_posterior_carry(bool seen) override { check(pm_engine_set_posterior_carry(eng_, seen ? 1 : 0)); }

 private:
  static void check(int rc) { if (rc) throw FatalError(std::string("GPU engine error: ") + pm_last_error() + "\n"); }
  pm_engine* eng_ = nullptr;
};

}  // namespace pmhost
