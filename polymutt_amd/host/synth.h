// synth.h -- synthetic pedigree templates and GLF dataset writer (see csrc/synth_core.h).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace pmhost {

struct SynthMember { int fa, mo, sex, pid; };   // family-local parent positions (-1 founder), sex, pid offset

// Template of family `fam` for a named shape, in Family::path order (founders first).
bool synth_shape(const std::string& shape, int fam, std::vector<SynthMember>& out);

// Writes dir/test.ped, test.dat, test.gif and one uncompressed GLF v3 file per person (section "1",
// dense positions 1..nsites) with the same sites pm_engine_synth generates on the device.
int synth_write_dataset(const std::string& dir, const std::string& shape, int nfam, int nsites, uint64_t seed, std::string& err);

}  // namespace pmhost
