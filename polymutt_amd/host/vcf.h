// vcf.h -- VCF text output, restating NucFamGenotypeLikelihood::OutputVCF / OutputVCF_denovo
// (src/NucFamGenotypeLikelihood.cpp:1751-1915) from engine results.
#pragma once
#include <cstdio>
#include <string>
#include "../../include/polymutt_engine.h"
#include "pedigree.h"

namespace pmhost {

struct VcfWriter {
  FILE* fh = nullptr;
  const Pedigree* ped = nullptr;
  std::string cmd;             // argv joined with single spaces + trailing space (main.cpp:159-164)
  double minMapQuality = 0;    // printed %f (CmdLinePar::minMapQuality is a double)
  int minTotalDepth = 0, maxTotalDepth = 0;
  double posterior = 0.5;
  bool gl_off = false, force_call = false, denovo = false;
  bool header_written = false;
  int chrom = PM_CHR_AUTO;

  // One OutputVCF(_denovo) call: writes the header on first use, then the record unless suppressed.
  void output(const std::string& label, int pos1, int refBase, const pm_site_result& r, const pm_geno_call* calls,
              const uint8_t* pl, const uint32_t* dm);
  void header();   // written by output() on first use; a sharded run's lead writes it once at the merge
  // The record text of an emitted site (r.emit == 1) appended to `out`, as output() writes it (no header, no I/O;
  // safe to call from several threads at once: the pipelined CLI formats a batch's records in parallel)
  void format(std::string& out, const std::string& label, int pos1, int refBase, const pm_site_result& r,
              const pm_geno_call* calls, const uint8_t* pl, const uint32_t* dm) const;

 private:
  bool singleNuclear() const;
  std::string line_;   // genotype columns of the record being written (reused)
};

}  // namespace pmhost
