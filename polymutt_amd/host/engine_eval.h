// engine_eval.h -- the HIP engine behind the driver's SiteEvaluator boundary (the product evaluator).
// There is no CPU fallback: without a usable HIP device pm_engine_create fails and the run stops.
//
// The pipelined CLI keeps several batches in flight: `engines` engine instances on the device (each with its own HIP
// stream and work buffers) take consecutive batches round-robin (pm_engine_submit), and the driver collects them
// in order (pm_engine_collect), so one batch's host-to-device copies overlap another's kernels.  Batch buffers are
// page-locked (pm_host_alloc), which makes those copies asynchronous.
//
// famlk[0]'s stale posterior state (pm_engine_set_posterior_carry) depends on whether any earlier site reached
// CalcPostProb; it changes only chrX/Y genotype posteriors (likelihoodONEKid's member sex).  So on
// autosomal sections batches run concurrently, and on chrX/Y/MT sections one at a time, each engine being told the
// state from the results collected so far before its batch is submitted.  The exception is --denovo: its
// posteriors do not read the carry (d_member_sex_before), so chrX/Y/MT batches stay concurrent there (in_flight()).
#pragma once
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <vector>
#include "../../include/polymutt_engine.h"
#include "driver.h"

namespace pmhost {

class EngineEvaluator : public SiteEvaluator {
 public:
  EngineEvaluator(const pm_pedigree& ped, const pm_params& par, int device, int batch, int engines = 1) {
    const auto t0 = std::chrono::steady_clock::now();
    const int k = std::max(1, std::min(engines, 8));
    for (int i = 0; i < k; i++) {
      pm_engine* e = nullptr;
      int rc = pm_engine_create(&ped, &par, device, batch, &e);
      if (rc) {
        for (auto* x : eng_) pm_engine_destroy(x);
        throw FatalError(std::string("GPU engine initialisation failed: ") + pm_last_error() + "\n");
      }
      eng_.push_back(e);
    }
    denovo_ = par.denovo != 0;
    if (getenv("PM_TIMING"))
      fprintf(stderr, "PM_TIMING engine create %.3f s (%d engines)\n",
              std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(), k);
  }
  ~EngineEvaluator() override {
    for (auto* e : eng_) pm_engine_destroy(e);
  }
  void begin_section(int chrom) override {
    for (auto* e : eng_) check(pm_engine_begin_section(e, chrom));
    chrom_ = chrom;
  }
  void run(int n, const uint8_t* pl, const uint32_t* dm, const uint8_t* ref, pm_site_result* res, pm_geno_call* calls,
           int* n_rows) override {
    check(pm_engine_set_posterior_carry(eng_[0], seen_ ? 1 : 0));
    int rc = pm_engine_run(eng_[0], n, pl, dm, ref, 0, res, calls, n_rows);
    if (rc == PM_EBRENT) throw stuck(eng_[0], *n_rows);
    check(rc);
    note(res, n);
  }
  void run_vcf(int n, int n_person, const uint8_t* pl, const uint8_t* ref, pm_site_result* res, pm_vcf_call* calls,
               int* n_rows) override {
    (void)n_person;
    check(pm_engine_set_posterior_carry(eng_[0], seen_ ? 1 : 0));
    int rc = pm_engine_run_vcf(eng_[0], n, pl, ref, res, calls, n_rows);
    if (rc == PM_EBRENT) throw stuck(eng_[0], *n_rows);
    check(rc);
    note(res, n);
  }
  void counters(pm_counters* out) override {   // the section totals summed over the engines
    memset(out, 0, sizeof(*out));
    for (auto* e : eng_) {
      pm_counters c;
      check(pm_engine_counters(e, &c));
      int64_t *d = (int64_t*)out, *s = (int64_t*)&c;
      for (size_t k = 0; k < sizeof(pm_counters) / sizeof(int64_t); k++) d[k] += s[k];
    }
  }
  void set_posterior_carry(bool seen) override {
    seen_ = seen;
    for (auto* e : eng_) check(pm_engine_set_posterior_carry(e, seen ? 1 : 0));
  }
  int in_flight() const override { return (chrom_ == PM_CHR_AUTO || denovo_) ? (int)eng_.size() : 1; }
  void submit(int n, const uint8_t* pl, const uint32_t* dm, const uint8_t* ref, pm_site_result* res, pm_geno_call* calls) override {
    pm_engine* e = eng_[next_ % eng_.size()];
    next_++;
    check(pm_engine_set_posterior_carry(e, seen_ ? 1 : 0));
    int rc = pm_engine_submit(e, n, pl, dm, ref);
    if (rc) { int r0; pm_engine_collect(e, res, calls, &r0); check(rc); }
    q_.push_back({e, n, res, calls});
  }
  int collect() override {
    Job j = q_.front();
    q_.pop_front();
    int rows = 0;
    int rc = pm_engine_collect(j.e, j.res, j.calls, &rows);
    if (rc == PM_EBRENT) throw stuck(j.e, rows);   // (the driver drains the writer first: no exit() with threads live)
    check(rc);
    note(j.res, j.n);
    return rows;
  }
  void* host_alloc(size_t bytes) override {
    void* p = nullptr;
    if (pm_host_alloc(bytes ? bytes : 1, &p) != PM_OK || !p) return SiteEvaluator::host_alloc(bytes);   // pageable fallback
    pinned_.push_back(p);
    return p;
  }
  void host_free(void* p) override {
    for (size_t i = 0; i < pinned_.size(); i++)
      if (pinned_[i] == p) { pinned_.erase(pinned_.begin() + i); pm_host_free(p); return; }
    SiteEvaluator::host_free(p);
  }

 private:
  struct Job { pm_engine* e; int n; pm_site_result* res; pm_geno_call* calls; };
  void note(const pm_site_result* res, int n) {   // CalcPostProb ran for a site: famlk[0]'s state is now set
    for (int i = 0; i < n && !seen_; i++) seen_ = res[i].emit != 0;
  }
  static void check(int rc) { if (rc) throw FatalError(std::string("GPU engine error: ") + pm_last_error() + "\n"); }
  // PM_EBRENT: the batch's sites before the first stuck one are complete (pm_engine_stuck_site), `rows` their rows
  static BrentError stuck(pm_engine* e, int rows) {
    int32_t k = 0;
    check(pm_engine_stuck_site(e, &k));
    return BrentError(k < 0 ? 0 : k, rows);
  }
  std::vector<pm_engine*> eng_;
  std::deque<Job> q_;
  std::vector<void*> pinned_;
  size_t next_ = 0;
  int chrom_ = PM_CHR_AUTO;
  bool denovo_ = false, seen_ = false;
};

}  // namespace pmhost
