// tests/native/cpu_polymutt.cpp -- TEST HARNESS ONLY.
// The product host driver (polymutt_amd/host) with the CPU oracle (oracle/pm_oracle.c) plugged in
// behind the SiteEvaluator boundary instead of the HIP engine.  Used by the CPU test suite to pin the
// host-side GLF reader, pedigree loader and VCF writer -- and the oracle itself -- against the
// reference's committed goldens.  Never shipped.
#include "oracle_eval.h"

int main(int argc, char** argv) { return pmhost::polymutt_main(argc, argv, nullptr, oracle_factory()); }
