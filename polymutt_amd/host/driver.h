// driver.h -- polymutt-compatible command line and section/site loop (src/main.cpp:57-627),
// batching sites into dense blocks for a SiteEvaluator (the HIP engine in the product binary).
#pragma once
#include <map>
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
  virtual void counters(pm_counters* out) = 0;
};

int default_io_threads(const Options& opt);

// Runs the whole analysis; returns the process exit code.
int run_polymutt(const Options& opt, const Pedigree& ped, SiteEvaluator& eval);

}  // namespace pmhost
