// vcf_input.h -- the --in_vcf path (src/PedVCF.cpp:43-164, src/FamilyLikelihoodSeq_VCF.cpp).
// Reads a VCF (plain or gzip) with per-sample PL (or GL) fields, maps samples to pedigree persons,
// evaluates every biallelic record with data on the SiteEvaluator (engine in vcf_mode: one Brent per
// record, posteriors at the minimiser) in batches, and writes the reference's modified VCF.
#pragma once
#include "driver.h"

namespace pmhost {

// Runs polymutt --in_vcf; returns the process exit code.  With comm->world > 1 the run is one shard: a
// byte slice of the records per rank, merged by rank 0 (vcf_input.cpp).
int run_polymutt_vcf(const Options& opt, const Pedigree& ped, SiteEvaluator& eval, const ShardComm* comm = nullptr);

}  // namespace pmhost
