// pedigree.cpp -- see pedigree.h.  Clean-room restatement of the reference's pedigree semantics.
#include "pedigree.h"
#include <zlib.h>
#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <cstring>
#include <cstdio>
#include <map>

namespace pmhost {

namespace {

std::string fmt(const char* f, ...) __attribute__((format(printf, 1, 2)));
std::string fmt(const char* f, ...) {
  char buf[4096];
  va_list ap; va_start(ap, f); vsnprintf(buf, sizeof(buf), f, ap); va_end(ap);
  return buf;
}

bool readLine(gzFile fh, std::string& line) {
  line.clear();
  int c;
  bool any = false;
  while ((c = gzgetc(fh)) != -1) {
    any = true;
    if (c == '\n') break;
    line.push_back((char)c);
  }
  return any;
}

std::vector<std::string> tokenize(const std::string& s, const char* seps) {
  std::vector<std::string> out;
  size_t i = 0, n = s.size();
  while (i < n) {
    while (i < n && strchr(seps, s[i]) && s[i]) i++;
    size_t j = i;
    while (j < n && !(strchr(seps, s[j]) && s[j])) j++;
    if (j > i) out.emplace_back(s.substr(i, j - i));
    i = j;
  }
  return out;
}

enum ColType { cAffection, cMarker, cTrait, cCovariate, cString, cSkip, cZygosity };

// Pedigree::TranslateSexCode, core/PedigreeLoader.cpp:574-598
int translateSex(const std::string& code, bool& failure) {
  failure = false;
  switch (code[0]) {
    case 'x': case 'X': case '?': return 0;
    case '1': case 'm': case 'M': return 1;
    case '2': case 'f': case 'F': return 2;
    default: {
      bool r = atoi(code.c_str()) != 0;   // the reference stores atoi() into a bool
      return r ? 1 : 0;
    }
  }
}

}  // namespace

// String::SlowCompare with NATURAL_ORDERING (core/StringBasics.cpp:24,431-448): compares up to and
// including the terminating NUL, case-insensitively; at the first difference a longer digit run wins.
int Pedigree::compareIds(const std::string& a, const std::string& b) {
  const char* x = a.c_str();
  const char* y = b.c_str();
  size_t len = a.size();
  for (size_t i = 0; i <= len; i++) {
    int d0 = toupper((unsigned char)x[i]) - toupper((unsigned char)y[i]);
    if (d0) {
      size_t d = i;
      while (isdigit((unsigned char)x[d]) && isdigit((unsigned char)y[d])) d++;
      if (isdigit((unsigned char)x[d])) return 1;
      if (isdigit((unsigned char)y[d])) return -1;
      return d0;
    }
    if (i >= b.size()) break;
  }
  return 0;
}

void Pedigree::load(const std::string& datFile, const std::string& pedFile) {
  // --- data file (PedigreeDescription::Load, core/PedigreeDescription.cpp:32-160) ---
  gzFile dat = gzopen(datFile.c_str(), "rb");
  if (!dat) throw FatalError("datFile open for input failed!\n");
  std::vector<ColType> cols;
  std::vector<std::string> colName;
  std::string line;
  bool done = false;
  while (!done && readLine(dat, line)) {
    auto t = tokenize(line, " \t\n\r\f");
    if (t.empty()) continue;
    if (t.size() == 1) {
      gzclose(dat);
      throw FatalError(fmt("Problem reading data file:\nItem #%zu (of type %s) has no name.", cols.size() + 1, t[0].c_str()));
    }
    switch (toupper((unsigned char)t[0][0])) {
      case 'A': cols.push_back(cAffection); colName.push_back(t[1]); break;
      case 'M': cols.push_back(cMarker); colName.push_back(t[1]); break;
      case 'T': cols.push_back(cTrait); colName.push_back(t[1]); break;
      case 'C': cols.push_back(cCovariate); colName.push_back(t[1]); break;
      case '$': cols.push_back(cString); colName.push_back(t[1]); break;
      case 'S': {
        int n = atoi(t[0].c_str() + 1);
        n = n > 0 ? n : 1;
        while (n--) { cols.push_back(cSkip); colName.push_back(""); }
        break;
      }
      case 'Z': cols.push_back(cZygosity); colName.push_back(""); break;
      case 'V': break;
      case 'E': done = true; break;
      default:
        gzclose(dat);
        throw FatalError(fmt("Problem in data file (line):\n%s\n", line.c_str()));
    }
  }
  gzclose(dat);
  int textCols = 5;
  for (auto c : cols) textCols += (c == cMarker) ? 2 : 1;

  // --- pedigree file (Pedigree::Load, core/PedigreeLoader.cpp:14-250) ---
  gzFile ped = gzopen(pedFile.c_str(), "rb");
  if (!ped) throw FatalError("pedFile open for input failed!\n");
  int lineNo = 0;
  while (readLine(ped, line)) {
    auto t = tokenize(line, " \t\n\r\f/");
    if (t.empty()) continue;
    if (compareIds(t[0], "end") == 0) break;
    lineNo++;
    if ((int)t.size() < textCols) {
      gzclose(ped);
      throw FatalError(fmt("Loading Pedigree...\n\nExpecting %d columns,\nbut read only %zu columns in line %d.\n",
                           textCols, t.size(), lineNo));
    }
    Person p;
    size_t field = 0;
    p.famid = t[field++]; p.pid = t[field++]; p.fatid = t[field++]; p.motid = t[field++];
    bool fail = false;
    p.sex = translateSex(t[field++], fail);
    for (size_t c = 0; c < cols.size(); c++) {
      switch (cols[c]) {
        case cMarker: field += 2; break;
        case cTrait: {
          const std::string& v = t[field++];
          if (colName[c] == "GLF_Index") {
            // strtod unless the value is the "-99.999" missing code; trailing junk -> missing
            double val = 6.66666e-66;
            if (v != "-99.999") {
              char* end = nullptr;
              double x = strtod(v.c_str(), &end);
              val = (end && *end) ? 6.66666e-66 : x;
            }
            p.glf_index = val;
          }
          break;
        }
        default: field++; break;
      }
    }
    persons.push_back(p);
  }
  gzclose(ped);

  // --- Pedigree::Sort (core/Pedigree.cpp:39-85) ---
  std::stable_sort(persons.begin(), persons.end(), [](const Person& a, const Person& b) {
    int r = compareIds(a.famid, b.famid);
    if (r) return r < 0;
    return compareIds(a.pid, b.pid) < 0;
  });
  bool problem = false;
  for (size_t i = 1; i < persons.size(); i++) {
    if (compareIds(persons[i - 1].famid, persons[i].famid) == 0 && compareIds(persons[i - 1].pid, persons[i].pid) == 0) {
      printf("Family %s: Person %s is duplicated\n", persons[i].famid.c_str(), persons[i].pid.c_str());
      problem = true;
    }
  }
  auto find = [&](const std::string& fam, const std::string& pid) -> int {
    size_t lo = 0, hi = persons.size();
    while (lo < hi) {
      size_t mid = (lo + hi) / 2;
      int r = compareIds(fam, persons[mid].famid);
      if (!r) r = compareIds(pid, persons[mid].pid);
      if (r == 0) return (int)mid;
      if (r < 0) hi = mid; else lo = mid + 1;
    }
    return -1;
  };
  for (size_t i = 0; i < persons.size(); i++) {
    Person& p = persons[i];
    int fa = find(p.famid, p.fatid), mo = find(p.famid, p.motid);
    if ((fa < 0) != (mo < 0)) {   // Person::CheckParents, core/PedigreePerson.cpp:90-126
      printf("Parent named %s for Person %s in Family %s is missing\n", fa < 0 ? p.fatid.c_str() : p.motid.c_str(),
             p.pid.c_str(), p.famid.c_str());
      problem = true;
      continue;
    }
    if (fa >= 0) {
      if (persons[fa].sex == 2 || persons[mo].sex == 1) { std::swap(fa, mo); std::swap(p.fatid, p.motid); }
      if (persons[fa].sex == 2 || persons[mo].sex == 1) {
        printf("Parental sex codes don't make sense for Person %s in Family %s\n", p.pid.c_str(), p.famid.c_str());
        problem = true;
      }
    }
    p.father = fa; p.mother = mo;
  }
  if (problem) throw FatalError("Please correct problems with pedigree structure\n");
  buildFamilies();
  flatten();
}

// Pedigree::MakeFamilies + Family::Family (core/Pedigree.cpp:122-143, core/PedigreeFamily.cpp:11-85)
void Pedigree::buildFamilies() {
  families.clear();
  size_t n = persons.size();
  for (size_t first = 0; first < n;) {
    size_t last = first;
    while (last < n && compareIds(persons[first].famid, persons[last].famid) == 0) last++;
    Family F;
    F.famid = persons[first].famid;
    F.first = (int)first;
    F.count = (int)(last - first);
    for (size_t i = first; i < last; i++)
      if (persons[i].founder()) { persons[i].traverse = F.founders++; F.path.push_back((int)i); }
      else persons[i].traverse = -1;
    F.generations = (F.count - F.founders) == 0 ? 1 : 2;
    int next = F.founders;
    while (next < F.count) {
      bool progress = false;
      for (size_t i = first; i < last; i++) {
        if (persons[i].traverse != -1) continue;
        int ft = persons[persons[i].father].traverse, mt = persons[persons[i].mother].traverse;
        if (ft >= 0 && mt >= 0) {
          progress = true;
          persons[i].traverse = next++;
          F.path.push_back((int)i);
          if (ft >= F.founders || mt >= F.founders) F.generations = 3;
        }
      }
      if (!progress) throw FatalError("Invalid pedigree structure.");
    }
    families.push_back(F);
    first = last;
  }
}

void Pedigree::flatten() {
  fam_start.clear(); fam_founders.clear(); fam_kind.clear(); peel_start.clear();
  sex.clear(); is_founder.clear(); father.clear(); mother.clear(); steps.clear(); column_pid.clear(); column_glf.clear();
  n_founders = male_founders = female_founders = 0;
  for (auto& F : families) {
    fam_start.push_back((int32_t)sex.size());
    fam_founders.push_back(F.founders);
    n_founders += F.founders;
    int kind = (F.count == F.founders) ? PM_FAM_FOUNDERS : (F.isNuclear() ? PM_FAM_NUCLEAR : PM_FAM_EXTENDED);
    fam_kind.push_back(kind);
    peel_start.push_back((int32_t)steps.size());
    std::vector<int> lsex;
    std::vector<std::pair<int, int>> lpar;
    std::vector<std::string> lpid;
    for (int j = 0; j < F.count; j++) {
      const Person& p = persons[F.path[j]];
      sex.push_back((int8_t)p.sex);
      is_founder.push_back(p.founder() ? 1 : 0);
      column_pid.push_back(p.pid);
      column_glf.push_back((int)p.glf_index);
      if (p.sex == 1 && p.founder()) male_founders++;     // PedigreeGLF::GetSexes, src/PedigreeGLF.cpp:99-116
      if (p.sex == 2 && p.founder()) female_founders++;
      lsex.push_back(p.sex);
      lpid.push_back(p.pid);
      lpar.emplace_back(p.founder() ? -1 : persons[p.father].traverse, p.founder() ? -1 : persons[p.mother].traverse);
      father.push_back(p.founder() ? -1 : fam_start.back() + persons[p.father].traverse);
      mother.push_back(p.founder() ? -1 : fam_start.back() + persons[p.mother].traverse);
    }
    if (kind != PM_FAM_FOUNDERS) {   // every family with offspring gets a schedule (FamilyLikelihoodSeq.cpp:32)
      F.peel = build_peeling_order(F.count, lsex, lpar, F.famid, lpid);
      steps.insert(steps.end(), F.peel.begin(), F.peel.end());
    }
  }
  fam_start.push_back((int32_t)sex.size());
  peel_start.push_back((int32_t)steps.size());
}

pm_pedigree Pedigree::view() const {
  pm_pedigree v;
  v.n_fam = (int32_t)families.size();
  v.n_person = (int32_t)sex.size();
  v.fam_start = fam_start.data();
  v.fam_founders = fam_founders.data();
  v.fam_kind = fam_kind.data();
  v.sex = sex.data();
  v.is_founder = is_founder.data();
  v.father = father.data();
  v.mother = mother.data();
  v.peel_start = peel_start.data();
  v.steps = steps.empty() ? nullptr : steps.data();
  v.n_founders = n_founders;
  v.male_founders = male_founders;
  v.female_founders = female_founders;
  return v;
}

// ---------------------------------------------------------------------------------------------
// Elston-Stewart peeling order (ES_Peeling, src/FamilyLikelihoodES.cpp:46-277), restated with
// std::vector queues.  Queue semantics: push_back / take front, exactly like IntArray Push/Delete(0).
std::vector<pm_peel_step> build_peeling_order(int n, const std::vector<int>& sex,
                                              const std::vector<std::pair<int, int>>& par,
                                              const std::string& famid, const std::vector<std::string>& pids) {
  std::vector<std::vector<int>> parents(n), offspring(n), spouses(n);
  std::map<std::pair<int, int>, int> couples;
  for (int i = 0; i < n; i++) {   // SetupConnections :46-78
    if (par[i].first < 0) continue;
    int fa = par[i].first, mo = par[i].second;
    parents[i] = {fa, mo};
    offspring[fa].push_back(i);
    offspring[mo].push_back(i);
    if (couples[{fa, mo}]++ == 0) { spouses[fa].push_back(mo); spouses[mo].push_back(fa); }
  }
  auto isLeaf = [&](int i) { return offspring[i].empty() && spouses[i].empty(); };
  auto isPeripheral = [&](int i) { return offspring[i].empty() && parents[i].empty() && spouses[i].size() == 1; };
  auto isFinal = [&](int i) { return parents[i].empty() && spouses[i].empty() && offspring[i].empty(); };
  auto isRoof = [&](int i) {
    if (spouses[i].size() != 1) return false;
    int s = spouses[i][0];
    return spouses[s].size() == 1 && parents[i].empty() && parents[s].empty() && offspring[i].size() == 1 && offspring[s].size() == 1;
  };
  auto findPair = [](const std::vector<std::pair<int, int>>& v, std::pair<int, int> p) {
    for (size_t k = 0; k < v.size(); k++)
      if ((v[k].first == p.first && v[k].second == p.second) || (v[k].first == p.second && v[k].second == p.first)) return (int)k;
    return -1;
  };
  auto removeOne = [](std::vector<int>& v, int x) {
    auto it = std::find(v.begin(), v.end(), x);
    if (it == v.end()) return false;
    v.erase(it);
    return true;
  };
  std::vector<int> leaf, peripheral;
  std::vector<std::pair<int, int>> roof;
  std::map<int, int> roofVisited;
  for (int i = 0; i < n; i++) {   // BuildInitialPeelable :80-114
    if (isLeaf(i)) { leaf.push_back(i); continue; }
    if (isRoof(i)) {
      int s = spouses[i][0];
      if (roofVisited[i] > 0 || roofVisited[s] > 0) continue;
      roof.push_back(sex[i] == 1 ? std::make_pair(i, s) : std::make_pair(s, i));
      roofVisited[i]++; roofVisited[s]++;
      continue;
    }
    if (isPeripheral(i)) { peripheral.push_back(i); continue; }
  }
  auto updateRoof = [&](int idx) {
    std::pair<int, int> c(idx, spouses[idx][0]);
    if (findPair(roof, c) >= 0) return;
    roof.push_back(c);
  };
  std::vector<pm_peel_step> out;
  int peeled = 0;
  bool done = false;
  for (;;) {   // BuildPeelingOrder :135-277
    if (leaf.empty() && roof.empty() && peripheral.empty()) break;
    if (done) break;
    while (!leaf.empty()) {
      int a = leaf.front(); leaf.erase(leaf.begin());
      peeled++;
      int fa = parents[a][0], mo = parents[a][1];
      out.push_back({1, a, -1, fa, mo});
      if (!removeOne(offspring[fa], a))
        throw FatalError("Peeling error for person " + pids[a] + " in family " + famid + "! Check pedigree structure!!\n");
      if (!removeOne(offspring[mo], a)) throw FatalError("Peeling leaf error!\n");
      parents[a].clear();
      if (isPeripheral(fa)) peripheral.push_back(fa);
      if (isPeripheral(mo)) peripheral.push_back(mo);
      int pos = findPair(roof, {fa, mo});
      if (pos > 0) roof.erase(roof.begin() + pos);   // `pos>0` as in the reference (:192-194)
      if (peeled == n - 1) done = true;
    }
    if (done) break;
    while (!peripheral.empty()) {
      int a = peripheral.front(); peripheral.erase(peripheral.begin());
      peeled++;
      if (spouses[a].size() > 1) throw FatalError("Peripheral parent can not have more than one spouses!\n");
      int to = spouses[a][0];
      out.push_back({2, a, -1, to, -1});
      if (!removeOne(spouses[to], a)) throw FatalError("No spouse can be found for person with PID of " + pids[a] + "!\n");
      spouses[a].clear();
      if (isFinal(to)) {
        if (peeled != n - 1)
          throw FatalError("Are there disconnected sub-pedigrees in family " + famid + "? Please move sub-pedigrees to separate families.\n");
        done = true;
        break;
      }
      if (isLeaf(to)) leaf.push_back(to);
      else if (isPeripheral(to)) peripheral.push_back(to);
      else if (isRoof(to)) updateRoof(to);
    }
    if (done) break;
    if (!leaf.empty() || !peripheral.empty()) continue;
    while (!roof.empty()) {
      std::pair<int, int> r = roof.front(); roof.erase(roof.begin());
      if (offspring[r.first].size() != 1 || offspring[r.second].size() != 1)
        throw FatalError("Roof can only have one offspring for peeling!\n");
      peeled += 2;
      int to = offspring[r.first][0];
      out.push_back({3, r.first, r.second, to, -1});
      parents[to].clear();
      offspring[r.first].clear();
      offspring[r.second].clear();
      if (isPeripheral(to)) peripheral.push_back(to);
      else if (isRoof(to)) updateRoof(to);
      else if (isFinal(to)) { done = true; break; }
    }
    if (done) break;
  }
  if (peeled < n - 1) throw FatalError("Are there inbreeding loops in the pedigree? It cannot handel inbreeding yet!\n");
  if (out.empty()) throw FatalError("Empty peeling order for family " + famid + "\n");
  return out;
}

}  // namespace pmhost
