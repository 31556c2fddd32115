// tests/native/cpu_polymutt.cpp -- TEST HARNESS ONLY.
// The product host driver (polymutt_amd/host) with the CPU oracle (oracle/pm_oracle.c) plugged in
// behind the SiteEvaluator boundary instead of the HIP engine.  Used by the CPU test suite to pin the
// host-side GLF reader, pedigree loader and VCF writer -- and the oracle itself -- against the
// reference's committed goldens.  Never shipped.
#include <cstdio>
#include <vector>
#include "../../polymutt_amd/host/blocks.h"
#include "../../polymutt_amd/host/driver.h"
#include "../../oracle/pm_oracle.h"

using namespace pmhost;

class OracleEvaluator : public SiteEvaluator {
 public:
  OracleEvaluator(const pm_pedigree& ped, const pm_params& par) : np_(ped.n_person) { ctx_ = pmo_create(&ped, &par); }
  ~OracleEvaluator() { pmo_destroy(ctx_); }
  void begin_section(int chrom) override { pmo_begin_section(ctx_, chrom); }
  void run(int n, const uint8_t* pl, const uint32_t* dm, const uint8_t* ref, pm_site_result* res, pm_geno_call* calls,
           int* n_rows) override {
    int rows = 0;
    for (int i = 0; i < n; i++) {
      int rc = pmo_site(ctx_, pl + (size_t)i * np_ * 10, dm + (size_t)i * np_, ref[i], &res[i], calls + (size_t)rows * np_);
      if (rc == PM_EBRENT) { printf("\nFATAL NUMERIC ERROR - ScalarMinimizer::Brent got stuck\n\n"); exit(1); }
      res[i].call_row = res[i].emit == 1 ? rows++ : -1;
    }
    *n_rows = rows;
  }
  void counters(pm_counters* out) override { pmo_counters(ctx_, out); }

 private:
  pmo_ctx* ctx_;
  int np_;
};

int main(int argc, char** argv) {
  try {
    Options opt = parse_command_line(argc, argv);
    Pedigree ped;
    ped.load(opt.datFile, opt.pedFile);
    if (!opt.blocksOut.empty()) {
      printf("%ld sites written\n", convert_glf_to_blocks(ped, opt.glfListFile, opt.blocksOut, default_io_threads(opt), opt.blockSites));
      return 0;
    }
    pm_pedigree v = ped.view();
    pm_params par = opt.params();
    OracleEvaluator ev(v, par);
    return run_polymutt(opt, ped, ev);
  } catch (const FatalError& e) {
    printf("\nFATAL ERROR - \n%s\n\n", e.what());
    return 1;
  }
}
