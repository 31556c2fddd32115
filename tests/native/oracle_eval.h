// tests/native/oracle_eval.h -- TEST HARNESS ONLY.
// The CPU oracle (oracle/pm_oracle.c) behind the product driver's SiteEvaluator boundary, in place of
// the HIP engine.  Never shipped.
#pragma once
#include <cstdio>
#include <cstdlib>
#ifdef _OPENMP
#include <omp.h>
#endif
#include "../../oracle/pm_oracle.h"
#include "../../polymutt_amd/host/driver.h"

class OracleEvaluator : public pmhost::SiteEvaluator {
 public:
  OracleEvaluator(const pm_pedigree& ped, const pm_params& par) : np_(ped.n_person) { ctx_ = pmo_create(&ped, &par); }
  ~OracleEvaluator() override { pmo_destroy(ctx_); }
  void begin_section(int chrom) override { pmo_begin_section(ctx_, chrom); }
  void run(int n, const uint8_t* pl, const uint32_t* dm, const uint8_t* ref, pm_site_result* res, pm_geno_call* calls,
           int* n_rows) override {
    int rows = 0;
    for (int i = 0; i < n; i++) {
      int rc = pmo_site(ctx_, pl + (size_t)i * np_ * 10, dm + (size_t)i * np_, ref[i], &res[i], calls + (size_t)rows * np_);
      if (rc == PM_EBRENT) throw pmhost::BrentError(i, rows);   // (the driver writes sites [0, i), then the FATAL text)
      res[i].call_row = res[i].emit == 1 ? rows++ : -1;
    }
    *n_rows = rows;
  }
  void counters(pm_counters* out) override { pmo_counters(ctx_, out); }
  void set_posterior_carry(bool seen) override { pmo_set_posterior_carry(ctx_, seen ? 1 : 0); }

 private:
  pmo_ctx* ctx_;
  int np_;
};

inline pmhost::EvaluatorFactory oracle_factory() {
  return [](const pm_pedigree& v, const pm_params& par, const pmhost::Options& opt) {
#ifdef _OPENMP
    if (opt.nthreads > 0) omp_set_num_threads(opt.nthreads);   // main.cpp:156 (default 1, :72)
#else
    (void)opt;
#endif
    return std::unique_ptr<pmhost::SiteEvaluator>(new OracleEvaluator(v, par));
  };
}
