// pedigree.h -- Merlin-format .dat/.ped loader with polyMutt's ordering, flattened to pm_pedigree.
//
// Mirrors the observable behaviour the reference relies on (core/Pedigree*.cpp, core/PedigreeFamily.cpp):
//   * persons sorted by (famid, pid), case-insensitive with natural digit ordering (core/StringBasics.cpp:431-470)
//   * families = runs of equal famid; Family::path = founders in sorted order, then descendants in
//     repeated sorted sweeps once both parents are placed (core/PedigreeFamily.cpp:11-85)
//   * generations / isNuclear() classification (core/PedigreeFamily.h:23-30)
//   * ES_Peeling schedule for non-nuclear families (src/FamilyLikelihoodES.cpp:46-277)
#pragma once
#include <string>
#include <vector>
#include <stdexcept>
#include "../../include/polymutt_engine.h"

namespace pmhost {

// Thrown for conditions where the reference calls error() (prints "FATAL ERROR" and exits 1).
struct FatalError : std::runtime_error { explicit FatalError(const std::string& m) : std::runtime_error(m) {} };
// Thrown where the reference calls numerror("ScalarMinimizer::Brent got stuck") (core/MathGold.cpp:98,175), which exits
// at the stuck site with every earlier record written (fflush per record, NucFamGenotypeLikelihood.cpp:1829): `valid`
// = the batch index of the first stuck site (its earlier sites' results are complete), `rows` = their genotype rows.
// The driver writes those records, then prints the reference's "FATAL NUMERIC ERROR" text and returns 1.
struct BrentError : std::runtime_error {
  int valid, rows;
  explicit BrentError(int valid_ = 0, int rows_ = 0)
      : std::runtime_error("ScalarMinimizer::Brent got stuck"), valid(valid_), rows(rows_) {}
};

struct Person {
  std::string famid, pid, fatid, motid;
  int sex = 0;                 // 0 unknown, 1 male, 2 female
  double glf_index = 6.66666e-66;   // trait "GLF_Index"; reference _NAN_ sentinel (core/Constant.h:16)
  int father = -1, mother = -1;     // indices into Pedigree::persons after sorting
  bool founder() const { return father < 0; }
  int traverse = -1;           // position in the family path
};

struct Family {
  std::string famid;
  int first = 0, count = 0, founders = 0, generations = 1;
  std::vector<int> path;       // person indices (global), founders first
  bool isNuclear() const { return generations == 2 && founders == 2; }
  std::vector<pm_peel_step> peel;   // every family with offspring (nuclear ones too)
};

class Pedigree {
 public:
  std::vector<Person> persons;
  std::vector<Family> families;

  void load(const std::string& datFile, const std::string& pedFile);

  // Flattened arrays (VCF column order = families in order, members in path order).
  std::vector<int32_t> fam_start, fam_founders, fam_kind, peel_start;
  std::vector<int8_t> sex, is_founder;
  std::vector<int32_t> father, mother;   // flattened person index of each parent, -1 for founders
  std::vector<pm_peel_step> steps;
  std::vector<std::string> column_pid;   // pid per flattened person
  std::vector<int> column_glf;           // (int) GLF_Index per flattened person
  int n_founders = 0, male_founders = 0, female_founders = 0;
  pm_pedigree view() const;

  static int compareIds(const std::string& a, const std::string& b);   // String::SlowCompare with natural ordering

 private:
  void buildFamilies();
  void flatten();
};

// ES_Peeling::SetupConnections + BuildInitialPeelable + BuildPeelingOrder for one family.
// `sex` and `parents` are family-local (path order).  Throws FatalError like the reference.
std::vector<pm_peel_step> build_peeling_order(int famSize, const std::vector<int>& sex,
                                              const std::vector<std::pair<int, int>>& parents,
                                              const std::string& famid, const std::vector<std::string>& pids);

}  // namespace pmhost
