// driver.h -- polymutt-compatible command line and section/site loop (src/main.cpp:57-627),
// batching sites into dense blocks for a SiteEvaluator (the HIP engine in the product binary).
#pragma once
#include <functional>
#include <map>
#include <memory>
#include <string>
#include <vector>
#include "../../include/polymutt_engine.h"
#include "pedigree.h"

namespace pmhost {

struct Options {
  std::string pedFile, datFile, glfListFile, vcfOutFile, vcfInFile, positionFile, chrs2process;
  std::string chrX = "X", chrY = "Y", MT = "MT";
  double posterior = 0.5, theta = 0.001, theta_indel = 0.0001, tstv = 2.0, precision = 0.0001;
  int minTotalDepth = 0, maxTotalDepth = 0, minMapQuality = 0, nthreads = 1;
  double minPS = 0;
  bool denovo = false, gl_off = false, quick_call = false, all_sites = false, force_call = false, exact_log10 = false;
  std::string numerics = "poly";
  double denovo_rate = 1.5e-08, denovo_tstv = 2.0, denovo_llr = 0.01;
  int device = 0, batch = 4096;
  int engines = 2;      // --engines: engine instances (HIP streams) with a batch in flight each (pipelined CLI)
  int io_threads = 0;   // GLF decode threads (0: min(16, hardware threads))
  std::string blocksIn, blocksOut;   // --in_blocks FILE (.pmb input in place of -g), --glf2blocks FILE (convert)
  int blockSites = 4096;
  std::string cmd;
  pm_params params() const;
};

// Parses argv the way ParameterList does for the flags polymutt declares (main.cpp:88-134).
// Throws FatalError on unknown options.
Options parse_command_line(int argc, char** argv);

// The compute backend behind the drop-in boundary.
class SiteEvaluator {
 public:
  virtual ~SiteEvaluator() {}
  virtual void begin_section(int chrom) = 0;
  virtual void run(int n, const uint8_t* pl, const uint32_t* dm, const uint8_t* ref, pm_site_result* res, pm_geno_call* calls,
                   int* n_rows) = 0;
  // vcf_mode: the genotype rows in their compact form (pm_engine_run_vcf); the default runs run() and narrows them
  virtual void run_vcf(int n, int n_person, const uint8_t* pl, const uint8_t* ref, pm_site_result* res, pm_vcf_call* calls,
                       int* n_rows);
  virtual void counters(pm_counters* out) = 0;
  // famlk[0]'s stale posterior state at a shard start (pm_engine_set_posterior_carry)
  virtual void set_posterior_carry(bool seen) = 0;
  // Batches in flight (the pipelined CLI): submit() starts a batch -- res / calls are filled by the matching
  // collect(), which returns its row count; batches are collected in submission order, and at most in_flight()
  // are outstanding.  The default runs the batch inside submit().
  virtual int in_flight() const { return 1; }
  // (a BrentError of the batch surfaces at its collect(), after the batches before it, as the engine's does)
  virtual void submit(int n, const uint8_t* pl, const uint32_t* dm, const uint8_t* ref, pm_site_result* res, pm_geno_call* calls) {
    int rows = 0, valid = -1;
    try {
      run(n, pl, dm, ref, res, calls, &rows);
    } catch (const BrentError& e) {
      valid = e.valid;
      rows = e.rows;
    }
    done_.push_back({rows, valid});
  }
  virtual int collect() {
    const std::pair<int, int> d = done_.front();
    done_.erase(done_.begin());
    if (d.second >= 0) throw BrentError(d.second, d.first);
    return d.first;
  }
  // Host memory for the batch buffers (the engine: page-locked, for asynchronous copies)
  virtual void* host_alloc(size_t bytes);
  virtual void host_free(void* p);

 private:
  std::vector<std::pair<int, int>> done_;   // (rows, first stuck site or -1) per submitted batch
};

// A run split over processes (one per GPU; polymutt_amd/launch.py): rank `rank` of `world` analyses a
// contiguous position range of every section.  `allgather` exchanges n int64 per rank (recv: world x n,
// rank-major); it is called the same number of times on every rank (once per section, once at the end).
struct ShardComm {
  int rank = 0, world = 1;
  std::function<void(const int64_t* send, int n, int64_t* recv)> allgather;
};

using EvaluatorFactory = std::function<std::unique_ptr<SiteEvaluator>(const pm_pedigree&, const pm_params&, const Options&)>;

int default_io_threads(const Options& opt);

// Runs the whole analysis; returns the process exit code.  With comm->world > 1 the run is one shard
// (run_polymutt_sharded).
int run_polymutt(const Options& opt, const Pedigree& ped, SiteEvaluator& eval, const ShardComm* comm = nullptr);

// The command line end to end (parse, pedigree, --glf2blocks, evaluator, run); FatalError -> the reference's
// "FATAL ERROR" text on stdout and exit code 1.
int polymutt_main(int argc, char** argv, const ShardComm* comm, const EvaluatorFactory& make);

}  // namespace pmhost
