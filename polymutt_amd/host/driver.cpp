// driver.cpp -- see driver.h.
#include "driver.h"
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <ctime>
#include "glf.h"
#include "ingest.h"
#include "blocks.h"
#include <atomic>
#include <memory>
#include <condition_variable>
#include <deque>
#include <exception>
#include <mutex>
#include <thread>
#include "vcf.h"
#include "vcf_input.h"

namespace pmhost {

pm_params Options::params() const {
  pm_params p;
  memset(&p, 0, sizeof(p));
  p.theta = theta; p.poly_tstv = tstv; p.precision = precision; p.posterior = posterior;
  p.min_total_depth = minTotalDepth; p.max_total_depth = maxTotalDepth; p.min_ps = minPS; p.min_map_quality = minMapQuality;
  p.denovo = denovo; p.denovo_mut_rate = denovo_rate; p.denovo_tstv = denovo_tstv; p.denovo_min_llr = denovo_llr;
  p.force_call = force_call; p.all_sites = all_sites; p.quick_call = quick_call; p.vcf_mode = vcfInFile.empty() ? 0 : 1;
  p.numerics = exact_log10 ? PM_NUM_EXACT : numerics == "exact" ? PM_NUM_EXACT : numerics == "poly" ? PM_NUM_POLY : PM_NUM_PRODUCT;
  return p;
}

Options parse_command_line(int argc, char** argv) {
  Options o;
  for (int a = 0; a < argc; a++) { o.cmd += argv[a]; o.cmd += " "; }
  struct Flag { const char* name; char kind; void* ptr; };   // kind: s string, d double, i int, b bool
  Flag longFlags[] = {
      {"in_vcf", 's', &o.vcfInFile}, {"theta", 'd', &o.theta}, {"indel_theta", 'd', &o.theta_indel},
      {"poly_tstv", 'd', &o.tstv}, {"chrX", 's', &o.chrX}, {"chrY", 's', &o.chrY}, {"MT", 's', &o.MT},
      {"denovo", 'b', &o.denovo}, {"rate_denovo", 'd', &o.denovo_rate}, {"tstv_denovo", 'd', &o.denovo_tstv},
      {"minLLR_denovo", 'd', &o.denovo_llr}, {"prec", 'd', &o.precision}, {"nthreads", 'i', &o.nthreads},
      {"chr2process", 's', &o.chrs2process}, {"minMapQuality", 'i', &o.minMapQuality}, {"minDepth", 'i', &o.minTotalDepth},
      {"maxDepth", 'i', &o.maxTotalDepth}, {"minPercSampleWithData", 'd', &o.minPS}, {"out_vcf", 's', &o.vcfOutFile},
      {"pos", 's', &o.positionFile}, {"all_sites", 'b', &o.all_sites}, {"gl_off", 'b', &o.gl_off},
      {"quick_call", 'b', &o.quick_call},
      // engine options (not in the reference)
      {"gpu", 'i', &o.device}, {"batch", 'i', &o.batch}, {"io_threads", 'i', &o.io_threads}, {"engines", 'i', &o.engines},
      {"in_blocks", 's', &o.blocksIn}, {"glf2blocks", 's', &o.blocksOut}, {"block_sites", 'i', &o.blockSites}, {"exact_log10", 'b', &o.exact_log10}, {"numerics", 's', &o.numerics},
  };
  auto assign = [](Flag& f, const char* v) {
    switch (f.kind) {
      case 's': *(std::string*)f.ptr = v; break;
      case 'd': *(double*)f.ptr = atof(v); break;
      case 'i': *(int*)f.ptr = atoi(v); break;
    }
  };
  for (int a = 1; a < argc; a++) {
    const char* s = argv[a];
    if (s[0] == '-' && s[1] == '-') {
      std::string name = s + 2, val;
      size_t eq = name.find('=');
      bool hasEq = eq != std::string::npos;
      if (hasEq) { val = name.substr(eq + 1); name = name.substr(0, eq); }
      bool found = false;
      for (auto& f : longFlags) {
        if (name != f.name) continue;
        found = true;
        if (f.kind == 'b') { *(bool*)f.ptr = true; break; }
        if (!hasEq) {
          if (a + 1 >= argc) throw FatalError(std::string("Missing value for option --") + name + "\n");
          val = argv[++a];
        }
        assign(f, val.c_str());
        break;
      }
      if (!found) throw FatalError(std::string("Unrecognized option --") + name + "\n");
    } else if (s[0] == '-' && s[1] && strchr("pdgc", s[1])) {
      const char* v = s[2] ? s + 2 : (a + 1 < argc ? argv[++a] : "");
      switch (s[1]) {
        case 'p': o.pedFile = v; break;
        case 'd': o.datFile = v; break;
        case 'g': o.glfListFile = v; break;
        case 'c': o.posterior = atof(v); break;
      }
    } else {
      throw FatalError(std::string("Unrecognized argument ") + s + "\n");
    }
  }
  if (!o.positionFile.empty()) { o.force_call = true; o.quick_call = false; o.all_sites = false; }   // main.cpp:151
  if (o.all_sites) o.quick_call = false;                                                            // main.cpp:153
  return o;
}

namespace {

}  // namespace

void* SiteEvaluator::host_alloc(size_t bytes) {
  void* p = malloc(bytes ? bytes : 1);
  if (!p) throw FatalError("out of host memory\n");
  return p;
}
void SiteEvaluator::host_free(void* p) { free(p); }

void SiteEvaluator::run_vcf(int n, int n_person, const uint8_t* pl, const uint8_t* ref, pm_site_result* res, pm_vcf_call* calls,
                            int* n_rows) {
  std::vector<uint32_t> dm((size_t)n * n_person, 0);
  std::vector<pm_geno_call> wide((size_t)n * n_person);
  auto narrow = [&](int rows) {   // (GQ <= 100, best <= 2 in vcf_mode: the device's 4-B form)
    for (size_t i = 0; i < (size_t)rows * n_person; i++) {
      pm_vcf_call c;
      c.best = (int8_t)wide[i].best; c.gq = (int8_t)wide[i].gq; c.label = wide[i].label; c.pad = 0;
      calls[i] = c;
    }
  };
  try {
    run(n, pl, dm.data(), ref, res, wide.data(), n_rows);
  } catch (const BrentError& e) {   // the rows of the sites before the stuck one are complete
    narrow(e.rows);
    throw;
  }
  narrow(*n_rows);
}

int default_io_threads(const Options& opt) {
  return opt.io_threads > 0 ? opt.io_threads : std::max(1, std::min(16, (int)std::thread::hardware_concurrency()));
}

namespace {

double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

void print_status(const Options& o) {   // abbreviated ParameterList::Status banner
  printf("\nThe following parameters are in effect:\n");
  printf("%30s : %s\n%30s : %s\n%30s : %s\n%30s : %g\n", "pedfile", o.pedFile.c_str(), "datfile", o.datFile.c_str(), "glfIndexFile",
         o.glfListFile.c_str(), "posterior cutoff", o.posterior);
  printf("%30s : theta=%g poly_tstv=%g prec=%g denovo=%s rate_denovo=%g minDepth=%d maxDepth=%d minMapQuality=%d out_vcf=%s\n\n",
         "Additional Options", o.theta, o.tstv, o.precision, o.denovo ? "ON" : "OFF", o.denovo_rate, o.minTotalDepth, o.maxTotalDepth,
         o.minMapQuality, o.vcfOutFile.c_str());
}

std::map<std::string, int> load_positions(const std::string& file) {   // LoadPositionFile, main.cpp:39-55
  std::map<std::string, int> m;
  FILE* fh = fopen(file.c_str(), "r");
  if (!fh) throw FatalError("Open position file " + file + " failed!\n");
  char line[65536];
  while (fgets(line, sizeof(line), fh)) {
    char a[4096], b[4096];
    if (sscanf(line, "%4095s %4095s", a, b) < 2) {
      if (sscanf(line, "%4095s", a) == 1) m[std::string(a) + ":"]++;
      continue;
    }
    m[std::string(a) + ":" + b]++;
  }
  fclose(fh);
  return m;
}

void print_summary(const std::string& label, int entries, const pm_counters& C, time_t t0) {   // main.cpp:596-620
  long total = 0;
  for (int k = 0; k < 5; k++) total += C.ref_base_counts[k];
  long other = C.tstvs1 + C.tstvs2 + C.tvs1tvs2;
  printf("Summary of reference -- %s\n", label.c_str());
  printf("Total Entry Count: %9d\n", entries);
  printf("Total Base Cout: %9ld\n", total);
  printf("Non-Polymorphic Count: %9ld\n", (long)C.homo_ref);
  printf("Transition Count: %9ld\n", (long)C.transitions);
  printf("Transversion Count: %9ld\n", (long)C.transversions);
  printf("Other Polymorphism Count: %9ld\n", other);
  printf("Filter counts:\n");
  printf("\tminMapQual %u\n", (unsigned)C.min_map_qual_filter);
  printf("\tminTotalDepth %u\n", (unsigned)C.min_total_depth_filter);
  printf("\tmaxTotalDepth %u\n", (unsigned)C.max_total_depth_filter);
  printf("Hard to call: %9ld\n", (long)C.nocall);
  printf("Skipped bases: %u\n", (unsigned)(entries - C.homo_ref - C.transitions - C.transversions - other));
  time_t t1; time(&t1);
  printf("Analysis ended on %s\n", ctime(&t1));
  printf("Running time is %u seconds\n\n", (unsigned)(t1 - t0));
}

// A closable blocking FIFO between the pipeline stages.
template <class T>
class Channel {
 public:
  void push(T v) {
    { std::lock_guard<std::mutex> l(mu_); q_.push_back(std::move(v)); }
    cv_.notify_one();
  }
  T pop() {
    std::unique_lock<std::mutex> l(mu_);
    cv_.wait(l, [&] { return !q_.empty(); });
    T v = std::move(q_.front());
    q_.pop_front();
    return v;
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<T> q_;
};

// One batch of sites: the dense block rows the engine reads (in the evaluator's host memory -- page-locked for the
// HIP engine, so its copies run asynchronously), the results and the genotype rows.
struct Batch {
  int n = 0, cap = 0, np = 0, rows = 0;
  SiteEvaluator* ev = nullptr;
  uint8_t *pl = nullptr, *ref = nullptr;
  uint32_t* dm = nullptr;
  pm_site_result* res = nullptr;
  pm_geno_call* calls = nullptr;
  std::vector<int> pos;
  Batch() = default;
  Batch(const Batch&) = delete;
  Batch& operator=(const Batch&) = delete;
  ~Batch() { release(); }
  void init(SiteEvaluator& e, int capacity, int nperson) {
    release();
    ev = &e; cap = capacity; np = nperson; n = 0;
    pl = (uint8_t*)e.host_alloc((size_t)cap * np * 10);
    dm = (uint32_t*)e.host_alloc((size_t)cap * np * 4);
    ref = (uint8_t*)e.host_alloc((size_t)cap);
    res = (pm_site_result*)e.host_alloc(sizeof(pm_site_result) * (size_t)cap);
    // (the genotype rows: pageable -- only the emitted rows are copied back, and pinning cap x n_person x 16 B per
    // batch would dominate start-up; malloc'd pages are touched only as rows arrive)
    calls = (pm_geno_call*)malloc(sizeof(pm_geno_call) * (size_t)cap * np);
    if (!calls) throw FatalError("out of host memory\n");
    pos.assign(cap, 0);
  }
  void release() {
    if (!ev) return;
    for (void* p : {(void*)pl, (void*)dm, (void*)ref, (void*)res}) ev->host_free(p);
    free(calls);
    pl = ref = nullptr; dm = nullptr; res = nullptr; calls = nullptr; ev = nullptr;
  }
};

std::map<std::string, int> parse_chr_selection(const std::string& s) {   // --chr2process (main.cpp:286-308)
  std::map<std::string, int> chrSel;
  size_t i = 0;
  while (i < s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    if (j > i) chrSel[s.substr(i, j - i)]++;
    i = j + 1;
  }
  return chrSel;
}

void copy_range(FILE* in, int64_t b, int64_t e, FILE* out) {
  std::vector<char> buf(1 << 20);
  if (fseek(in, (long)b, SEEK_SET) != 0) throw FatalError("VCF shard merge: seek failed\n");
  while (b < e) {
    const size_t want = (size_t)std::min<int64_t>(e - b, (int64_t)buf.size());
    const size_t got = fread(buf.data(), 1, want, in);
    if (got != want) throw FatalError("VCF shard merge: short read\n");
    fwrite(buf.data(), 1, got, out);
    b += (int64_t)got;
  }
}

}  // namespace

// One shard of a multi-process run: rank R of N analyses the sites of every section whose
// 0-based position lies in [maxPosition * R / N, maxPosition * (R + 1) / N) (the last rank: to the end),
// writes their records to <out_vcf>.part<R>, and at each section end exchanges one small vector per rank
// (the section counters of main.cpp:264-282, the entry count, how many sites reached OutputVCF, the byte
// range of its records).  Rank 0 prints the summed section summary (main.cpp:596-619) and finally
// concatenates the parts in (section, rank) order behind the header, which the reference writes lazily on
// the first OutputVCF call.
//
// Cross-shard state: famlk[0]'s stale member sex (pm_engine_set_posterior_carry) depends on whether any
// earlier site in run order reached CalcPostProb.  Earlier sections are known to every rank; for its own
// section range rank R > 0 assumes an earlier shard emitted something, and after the exchange, when that
// guess was wrong and the shard has a record, re-runs the shard's first recorded site with the true state
// and writes that record to <out_vcf>.part<R>.fix<section>, which the merge puts in place of the first one.
int run_polymutt_sharded(const Options& opt, const Pedigree& ped, SiteEvaluator& eval, const ShardComm& comm, SiteStream& src) {
  const int R = comm.rank, N = comm.world;
  const bool lead = R == 0;
  if (!opt.positionFile.empty()) throw FatalError("--pos runs cannot be sharded over several processes\n");
  const std::string part = opt.vcfOutFile + ".part" + std::to_string(R);
  FILE* fh = fopen(part.c_str(), "w+b");
  if (!fh) throw FatalError("vcfOutFile can not be opened for output!\n");
  VcfWriter W;
  W.fh = fh; W.ped = &ped; W.cmd = opt.cmd; W.minMapQuality = opt.minMapQuality; W.minTotalDepth = opt.minTotalDepth;
  W.maxTotalDepth = opt.maxTotalDepth; W.posterior = opt.posterior; W.gl_off = opt.gl_off; W.force_call = opt.force_call;
  W.denovo = opt.denovo;
  W.header_written = true;   // parts hold records only
  std::map<std::string, int> chrSel = parse_chr_selection(opt.chrs2process);
  const size_t chrSelCount = chrSel.size();
  time_t t0; time(&t0);
  if (lead) printf("Analysis started on %s\n", ctime(&t0));
  const int np = (int)ped.column_pid.size();
  Batch B;
  B.init(eval, opt.batch > 0 ? opt.batch : 4096, np);
  enum { K_ENTRIES = 16, K_OUT, K_REC, K_START, K_END, K_FIRST_END, K_STUCK, K };
  // A Brent stuck at ITMAX (core/MathGold.cpp:98,175) ends the reference's run at that site, every earlier record
  // written, no summary for the section: the stuck shard writes its records before the site, the exchange tells every
  // rank, and the merge takes this section's parts of the shards up to the first stuck one only.
  int stuck_rank = -1;
  bool earlier = false;        // a site of an earlier section (any shard) reached CalcPostProb
  int64_t outputs = 0;         // OutputVCF calls over all shards: the header exists iff > 0
  std::vector<std::vector<int64_t>> secs;   // lead: every section's exchange (N x K)
  std::vector<std::vector<char>> fixes;     // lead: per section and rank, a .fix record replaces the first one
  size_t chrDone = 0;
  std::vector<int> wpos(src.window()), rowOf(src.window());
  std::vector<uint8_t> wref(src.window());
  while (src.nextSection()) {
    if (!chrSel.empty() && chrDone >= chrSelCount) break;
    const std::string label = src.label();
    if (!chrSel.empty() && chrSel[label] < 1) continue;
    const int chrom = label == opt.chrX ? PM_CHR_X : label == opt.chrY ? PM_CHR_Y : label == opt.MT ? PM_CHR_MT : PM_CHR_AUTO;
    chrDone++;
    eval.begin_section(chrom);
    W.chrom = chrom;
    const int64_t mp = src.maxPosition();
    const int64_t lo = mp * R / N, hi = (R == N - 1) ? INT64_MAX : mp * (R + 1) / N;
    const bool guess = earlier || R > 0;
    eval.set_posterior_carry(guess);
    // Block input seeks straight to the shard's first block (blocks.h index); GLF input cannot be seeked, so a
    // GLF shard reads and drops the sites below lo (multi-GPU runs should convert with --glf2blocks first).
    const long blocks0 = src.blocksRead();
    const bool seeked = N > 1 && src.seek(lo, hi);
    int64_t entries = 0, n_out = 0, n_rec = 0, first_end = -1;
    const int64_t start = ftell(fh);
    std::vector<uint8_t> fpl((size_t)np * 10);
    std::vector<uint32_t> fdm(np);
    uint8_t fref = 0;
    int fpos = 0;
    bool past = false, stuck = false;
    auto flush = [&]() {
      if (B.n == 0) return;
      int rows = 0, nv = B.n;
      try {
        eval.run(B.n, B.pl, B.dm, B.ref, B.res, B.calls, &rows);
      } catch (const BrentError& e) {   // the sites before the stuck one are complete
        nv = e.valid;
        stuck = true;
      }
      for (int i = 0; i < nv; i++) {
        const pm_site_result& r = B.res[i];
        if (!r.emit) continue;
        n_out++;
        const uint8_t* pl = B.pl + (size_t)i * np * 10;
        const uint32_t* dm = B.dm + (size_t)i * np;
        W.output(label, B.pos[i], B.ref[i], r, r.call_row >= 0 ? B.calls + (size_t)r.call_row * np : nullptr, pl, dm);
        if (r.emit != 1) continue;
        if (n_rec++ == 0) {   // the shard's first record: keep its site for a possible re-run
          first_end = ftell(fh);
          memcpy(fpl.data(), pl, fpl.size());
          memcpy(fdm.data(), dm, fdm.size() * sizeof(uint32_t));
          fref = B.ref[i];
          fpos = B.pos[i];
        }
      }
      B.n = 0;
    };
    for (;;) {
      const int got = src.nextSites(std::min(src.window(), B.cap - B.n), wpos.data(), wref.data());
      if (got > 0) entries = mp;
      for (int k = 0; k < got; k++) {
        rowOf[k] = -1;
        if (wpos[k] < lo) continue;
        if (wpos[k] >= hi) { past = true; continue; }
        const int i = B.n++;
        B.pos[i] = wpos[k] + 1;
        B.ref[i] = wref[k];
        rowOf[k] = i;
      }
      src.fill(rowOf.data(), B.pl, B.dm);
      if (B.n == B.cap) flush();
      if (stuck || past || src.ended()) break;
    }
    if (!stuck) flush();
    if (past && !stuck) src.skipSection();   // the rest of the section belongs to later shards
    if (getenv("PM_BLOCK_STATS") && blocks0 >= 0)
      fprintf(stderr, "PM_BLOCK_STATS shard %d section %s: blocks read %ld%s\n", R, label.c_str(), src.blocksRead() - blocks0,
              seeked ? " (seeked)" : "");
    pm_counters C;
    eval.counters(&C);
    static_assert(sizeof(pm_counters) == 16 * sizeof(int64_t), "counter layout");
    std::vector<int64_t> send(K), recv((size_t)N * K);
    memcpy(send.data(), &C, sizeof(C));
    send[K_ENTRIES] = entries; send[K_OUT] = n_out; send[K_REC] = n_rec;
    send[K_START] = start; send[K_END] = ftell(fh); send[K_FIRST_END] = first_end; send[K_STUCK] = stuck;
    comm.allgather(send.data(), K, recv.data());
    for (int q = N - 1; q >= 0; q--)
      if (recv[(size_t)q * K + K_STUCK]) stuck_rank = q;
    const int last_q = stuck_rank >= 0 ? stuck_rank : N - 1;   // this section's parts that reach the output
    auto needs_fix = [&](int q) {   // shard q's first record was formatted with the wrong famlk[0] state
      bool truth = earlier;
      for (int p = 0; p < q; p++) truth = truth || recv[(size_t)p * K + K_OUT] > 0;
      return recv[(size_t)q * K + K_REC] > 0 && truth != (earlier || q > 0);
    };
    if (R <= last_q && needs_fix(R)) {
      fprintf(stderr, "shard %d: section %s: first record re-run with famlk[0] posterior state %s\n", R, label.c_str(),
              (earlier || R > 0) ? "unset" : "set");
      eval.set_posterior_carry(!(earlier || R > 0));
      pm_site_result r1;
      std::vector<pm_geno_call> c1(np);
      int rows = 0;
      eval.run(1, fpl.data(), fdm.data(), &fref, &r1, c1.data(), &rows);
      char* buf = nullptr;
      size_t len = 0;
      FILE* ms = open_memstream(&buf, &len);
      VcfWriter W1 = W;
      W1.fh = ms;
      W1.output(label, fpos, fref, r1, r1.call_row >= 0 ? c1.data() : nullptr, fpl.data(), fdm.data());
      fclose(ms);
      FILE* fx = fopen((part + ".fix" + std::to_string(secs.size())).c_str(), "wb");
      if (!fx) { free(buf); throw FatalError("vcfOutFile can not be opened for output!\n"); }
      fwrite(buf, 1, len, fx);
      fclose(fx);
      free(buf);
    }
    if (lead) {
      pm_counters S;
      memset(&S, 0, sizeof(S));
      int64_t* s = (int64_t*)&S;
      int64_t ent = 0;
      std::vector<char> fx(N);
      for (int q = 0; q < N; q++) {
        for (int k = 0; k < 16; k++) s[k] += recv[(size_t)q * K + k];
        ent = std::max(ent, recv[(size_t)q * K + K_ENTRIES]);
        fx[q] = q <= last_q && needs_fix(q);
      }
      if (stuck_rank < 0) print_summary(label, (int)ent, S, t0);
      secs.push_back(recv);
      fixes.push_back(fx);
    } else secs.emplace_back();   // keeps the section numbering of the .fix files
    for (int q = 0; q <= last_q; q++) {
      outputs += recv[(size_t)q * K + K_OUT];
      earlier = earlier || recv[(size_t)q * K + K_OUT] > 0;
    }
    if (stuck_rank >= 0) break;
  }
  fflush(fh);
  fclose(fh);
  {   // every shard's part and fixes are complete before the lead concatenates them
    int64_t one = 1;
    std::vector<int64_t> all(N);
    comm.allgather(&one, 1, all.data());
  }
  if (!lead) return stuck_rank >= 0 ? 1 : 0;   // (the lead prints the FATAL text once)
  FILE* out = fopen(opt.vcfOutFile.c_str(), "w");
  if (!out) throw FatalError("vcfOutFile can not be opened for output!\n");
  if (outputs > 0) { W.fh = out; W.header_written = false; W.header(); }
  std::vector<FILE*> parts(N);
  for (int q = 0; q < N; q++) {
    parts[q] = fopen((opt.vcfOutFile + ".part" + std::to_string(q)).c_str(), "rb");
    if (!parts[q]) throw FatalError("VCF shard merge: a shard's part file is missing\n");
  }
  for (size_t s = 0; s < secs.size(); s++)
    for (int q = 0; q < N; q++) {
      if (stuck_rank >= 0 && s + 1 == secs.size() && q > stuck_rank) break;   // after the stuck site: never written
      const int64_t* v = secs[s].data() + (size_t)q * K;
      if (fixes[s][q]) {
        const std::string fxp = opt.vcfOutFile + ".part" + std::to_string(q) + ".fix" + std::to_string(s);
        FILE* fx = fopen(fxp.c_str(), "rb");
        if (!fx) throw FatalError("VCF shard merge: a shard's fix record is missing\n");
        fseek(fx, 0, SEEK_END);
        copy_range(fx, 0, ftell(fx), out);
        fclose(fx);
        remove(fxp.c_str());
        copy_range(parts[q], v[K_FIRST_END], v[K_END], out);
      } else copy_range(parts[q], v[K_START], v[K_END], out);
    }
  for (int q = 0; q < N; q++) {
    fclose(parts[q]);
    remove((opt.vcfOutFile + ".part" + std::to_string(q)).c_str());
  }
  fclose(out);
  if (stuck_rank >= 0) throw BrentError();
  return 0;
}

int run_polymutt(const Options& opt, const Pedigree& ped, SiteEvaluator& eval, const ShardComm* comm) {
  const bool sharded = comm && (comm->world > 1 || comm->allgather);   // (world 1 with an exchange: the shard protocol)
  if (!sharded || comm->rank == 0) print_status(opt);
  if (opt.vcfInFile == opt.vcfOutFile) throw FatalError("Input and output VCF files are the same!\n");
  if (opt.pedFile.empty()) throw FatalError("pedFile not provided for input!\n");
  if (opt.glfListFile.empty() && opt.vcfInFile.empty() && opt.blocksIn.empty())
    throw FatalError("glfListFile or input VCF file not provided for input!\n");
  if (opt.vcfOutFile.empty()) throw FatalError("vcfOutFile not provided for output!\n");
  if (!opt.vcfInFile.empty()) {   // main.cpp:238-246
    return run_polymutt_vcf(opt, ped, eval, sharded ? comm : nullptr);
  }
  if (opt.denovo && opt.denovo_llr < 0) throw FatalError("denovo_min_LLR can only be greater than 0 !\n");

  std::map<std::string, int> positionMap;
  if (!opt.positionFile.empty()) positionMap = load_positions(opt.positionFile);

  const double t_open0 = now_s();
  std::unique_ptr<SiteStream> srcp;
  if (!opt.blocksIn.empty()) {   // dense indexed blocks (blocks.h)
    auto* b = new BlockSiteSource;
    srcp.reset(b);
    b->open(opt.blocksIn, (int)ped.column_pid.size(), default_io_threads(opt));
  } else {   // PedigreeGLF with parallel decode (ingest.h)
    auto* g = new ParallelSiteSource;
    srcp.reset(g);
    // sites per merge window (PM_GLF_WINDOW): 4096 measured best of 512-16384 (profiles/r05v_glf_window.json)
    const char* ew = getenv("PM_GLF_WINDOW");
    g->open(ped, opt.glfListFile, default_io_threads(opt), ew ? std::max(64, atoi(ew)) : 4096);
  }
  SiteStream& src = *srcp;
  if (getenv("PM_TIMING")) fprintf(stderr, "PM_TIMING open inputs %.3f s\n", now_s() - t_open0);
  if (sharded) return run_polymutt_sharded(opt, ped, eval, *comm, src);
  FILE* vcf = fopen(opt.vcfOutFile.c_str(), "w");
  if (!vcf) throw FatalError("vcfOutFile can not be opened for output!\n");

  VcfWriter W;
  W.fh = vcf; W.ped = &ped; W.cmd = opt.cmd; W.minMapQuality = opt.minMapQuality; W.minTotalDepth = opt.minTotalDepth;
  W.maxTotalDepth = opt.maxTotalDepth; W.posterior = opt.posterior; W.gl_off = opt.gl_off; W.force_call = opt.force_call;
  W.denovo = opt.denovo;

  std::map<std::string, int> chrSel = parse_chr_selection(opt.chrs2process);
  const size_t chrSelCount = chrSel.size();
  time_t t0; time(&t0);
  printf("Analysis started on %s\n", ctime(&t0));

  const int np = (int)ped.column_pid.size();
  Batch B;   // (the serial loop's buffer; the pipeline has its own pool)
  int out_cnt = 0;
  size_t chrDone = 0;
  double t_ingest = 0, t_eval = 0, t_out = 0;   // PM_TIMING=1: host-side breakdown on stderr
  struct TimingReport {
    double &a, &b, &c;
    ~TimingReport() {
      if (getenv("PM_TIMING")) fprintf(stderr, "PM_TIMING ingest %.3f s, engine %.3f s, vcf %.3f s\n", a, b, c);
    }
  } timing_report{t_ingest, t_eval, t_out};

  auto chrom_of = [&](const std::string& label) {
    return label == opt.chrX ? PM_CHR_X : label == opt.chrY ? PM_CHR_Y : label == opt.MT ? PM_CHR_MT : PM_CHR_AUTO;
  };
  if (!opt.force_call && !getenv("PM_SERIAL")) {
    // Three stages: ingest (producer thread: GLF decode + merge, or parallel block reads,
    // into page-locked batch buffers) -> engine (this thread: batches submitted in order to the evaluator, which
    // keeps up to in_flight() of them running on separate engines / HIP streams, and collected in order) -> VCF
    // writer thread (the batch's records formatted in parallel and written in order, then the section summary).
    // in_flight() + 3 batch buffers rotate, so the ingest of later batches, the copies and kernels of several
    // batches and the formatting of earlier ones overlap.  Output order is the serial one.
    // (--pos runs stop after the listed sites, main.cpp:593; they take the serial loop below.)
    enum { M_SECTION, M_BATCH, M_END, M_DONE };
    struct Msg { int kind; Batch* b; std::string label; int chrom; int entries; pm_counters C; };
    const int cap = opt.batch > 0 ? opt.batch : 4096;
    std::vector<std::unique_ptr<Batch>> pool;
    Channel<Batch*> freeq;
    for (int i = 0; i < 3 + std::max(1, eval.in_flight()); i++) {
      pool.emplace_back(new Batch);
      pool.back()->init(eval, cap, np);
      freeq.push(pool.back().get());
    }
    Channel<Msg> toEngine, toWriter;
    std::atomic<bool> abort{false};
    std::exception_ptr perr, eerr, werr;
    // PM_TIMING: wall clock of the pipeline (since the inputs were opened): first batch handed on, ingest done, end
    double w_first = 0, w_ingest = 0, w_sec = 0, w_sites1 = 0, w_fill1 = 0;
    struct WallReport {
      double t0, &first, &ingest;
      ~WallReport() {
        if (getenv("PM_TIMING"))
          fprintf(stderr, "PM_TIMING wall: first batch %.3f s, ingest done %.3f s, end %.3f s\n", first - t0, ingest - t0, now_s() - t0);
        if (getenv("PM_TIMING") && sec > 0)
          fprintf(stderr, "PM_TIMING first window: section %.3f s, sites %.3f s, fill %.3f s\n", sec - t0, sites1 - t0, fill1 - t0);
      }
      double &sec, &sites1, &fill1;
    } wall_report{t_open0, w_first, w_ingest, w_sec, w_sites1, w_fill1};
    std::thread producer([&] {
      try {
        size_t done = 0;
        std::vector<int> wpos(src.window()), rowOf(src.window());
        std::vector<uint8_t> wref(src.window());
        while (!abort && src.nextSection()) {
          if (!chrSel.empty() && done >= chrSelCount) break;
          const std::string label = src.label();
          if (!chrSel.empty() && chrSel[label] < 1) continue;   // the next section's skip consumes this one
          const int chrom = chrom_of(label);
          if (w_sec == 0) w_sec = now_s();
          done++;
          toEngine.push({M_SECTION, nullptr, label, chrom, 0, {}});
          int entries = 0;
          Batch* b = freeq.pop();
          b->n = 0;
          while (!abort) {
            const double ti = now_s();
            const int want = std::min(src.window(), b->cap - b->n);
            const int got = src.nextSites(want, wpos.data(), wref.data());
            if (w_sites1 == 0) w_sites1 = now_s();
            if (got > 0 && entries == 0) entries = src.maxPosition();
            for (int k = 0; k < got; k++) {
              const int i = b->n++;
              b->pos[i] = wpos[k] + 1;
              b->ref[i] = wref[k];
              rowOf[k] = i;
            }
            src.fill(rowOf.data(), b->pl, b->dm);
            if (w_fill1 == 0) w_fill1 = now_s();
            t_ingest += now_s() - ti;
            if (b->n == b->cap) {
              if (w_first == 0) w_first = now_s();
              toEngine.push({M_BATCH, b, label, chrom, 0, {}});
              b = freeq.pop();
              b->n = 0;
            }
            if (src.ended()) break;
          }
          if (b->n > 0) {
            if (w_first == 0) w_first = now_s();
            toEngine.push({M_BATCH, b, label, chrom, 0, {}});
          } else freeq.push(b);
          toEngine.push({M_END, nullptr, label, chrom, entries, {}});
        }
      } catch (...) {
        perr = std::current_exception();
      }
      w_ingest = now_s();
      toEngine.push({M_DONE, nullptr, "", 0, 0, {}});
    });
    std::thread writer([&] {
      // a batch's records are formatted in parallel (VcfWriter::format) into per-chunk buffers, then written in order
      TaskPool fmt_pool(default_io_threads(opt));
      std::vector<std::string> chunks;
      std::vector<int> recs;
      for (;;) {
        Msg m = toWriter.pop();
        if (m.kind == M_DONE) break;
        try {
          if (m.kind == M_BATCH && !werr) {
            const double t1 = now_s();
            W.chrom = m.chrom;
            const Batch& b = *m.b;
            recs.clear();
            bool any = false;
            for (int i = 0; i < b.n; i++) {
              any = any || b.res[i].emit != 0;   // (a suppressed de novo record writes the header too, :1868)
              if (b.res[i].emit == 1) recs.push_back(i);
            }
            if (any && !W.header_written) W.header();
            const int nc = std::min((int)recs.size(), 4 * fmt_pool.threads());
            if ((int)chunks.size() < nc) chunks.resize(nc);
            auto format_chunk = [&](int c) {
              std::string& out = chunks[c];
              out.clear();
              for (size_t k = (size_t)c * recs.size() / nc; k < (size_t)(c + 1) * recs.size() / nc; k++) {
                const int i = recs[k];
                const pm_site_result& r = b.res[i];
                W.format(out, m.label, b.pos[i], b.ref[i], r, b.calls + (size_t)r.call_row * np, b.pl + (size_t)i * np * 10,
                         b.dm + (size_t)i * np);
              }
            };
            if (nc > 1) fmt_pool.run(nc, format_chunk);
            else if (nc == 1) format_chunk(0);
            for (int c = 0; c < nc; c++) fwrite(chunks[c].data(), 1, chunks[c].size(), vcf);
            if (nc) fflush(vcf);
            t_out += now_s() - t1;
          } else if (m.kind == M_END && !werr) {
            print_summary(m.label, m.entries, m.C, t0);
            fflush(vcf);
          }
        } catch (...) {
          werr = std::current_exception();
          abort = true;
        }
        if (m.kind == M_BATCH) freeq.push(m.b);
      }
    });
    std::deque<Msg> inflight;   // submitted, not yet collected (submission order)
    auto retire = [&]() {       // collect the oldest batch and hand it to the writer
      Msg m = std::move(inflight.front());
      inflight.pop_front();
      const double te = now_s();
      try {
        m.b->rows = eval.collect();
      } catch (const BrentError& e) {   // the writer gets the sites before the stuck one, then the run ends
        m.b->n = e.valid;
        m.b->rows = e.rows;
        toWriter.push(std::move(m));
        throw;
      } catch (...) {
        freeq.push(m.b);
        throw;
      }
      t_eval += now_s() - te;
      toWriter.push(std::move(m));
    };
    for (;;) {   // engine stage
      Msg m = toEngine.pop();
      if (m.kind == M_DONE) {
        try {
          while (!inflight.empty() && !eerr) retire();
        } catch (...) {
          eerr = std::current_exception();
          abort = true;
        }
        for (auto& x : inflight) freeq.push(x.b);
        inflight.clear();
        toWriter.push(m);
        break;
      }
      if (eerr) {   // draining after an engine error
        if (m.kind == M_BATCH) freeq.push(m.b);
        continue;
      }
      try {
        if (m.kind == M_SECTION) {
          while (!inflight.empty()) retire();
          eval.begin_section(m.chrom);
        } else if (m.kind == M_BATCH) {
          while (!inflight.empty() && (int)inflight.size() >= eval.in_flight()) retire();
          const double te = now_s();
          Batch& b = *m.b;
          eval.submit(b.n, b.pl, b.dm, b.ref, b.res, b.calls);
          t_eval += now_s() - te;
          inflight.push_back(std::move(m));
        } else if (m.kind == M_END) {
          while (!inflight.empty()) retire();
          eval.counters(&m.C);
          toWriter.push(m);
        }
      } catch (...) {
        eerr = std::current_exception();
        abort = true;
        if (m.kind == M_BATCH) freeq.push(m.b);
        for (auto& x : inflight) freeq.push(x.b);
        inflight.clear();
      }
    }
    producer.join();
    writer.join();
    for (auto* e : {&eerr, &perr, &werr})
      if (*e) std::rethrow_exception(*e);
    fclose(vcf);
    return 0;
  }

  B.init(eval, opt.batch > 0 ? opt.batch : 4096, np);
  while (src.nextSection()) {
    if (!chrSel.empty() && chrDone >= chrSelCount) break;
    const std::string label = src.label();
    if (!chrSel.empty() && chrSel[label] < 1) continue;   // the next section's skip consumes this one
    const int chrom = chrom_of(label);
    eval.begin_section(chrom);
    W.chrom = chrom;
    chrDone++;
    int entries = 0;
    bool stop = false;

    auto flush = [&]() {
      if (B.n == 0) return;
      int rows = 0, nv = B.n;
      const double t0 = now_s();
      std::exception_ptr stuck;
      try {
        eval.run(B.n, B.pl, B.dm, B.ref, B.res, B.calls, &rows);
      } catch (const BrentError& e) {   // write the sites before the stuck one, then end the run
        nv = e.valid;
        stuck = std::current_exception();
      }
      const double t1 = now_s();
      t_eval += t1 - t0;
      for (int i = 0; i < nv && !stop; i++) {
        const pm_site_result& r = B.res[i];
        if (!r.emit) continue;
        W.output(label, B.pos[i], B.ref[i], r, r.call_row >= 0 ? B.calls + (size_t)r.call_row * np : nullptr, B.pl + (size_t)i * np * 10,
                 B.dm + (size_t)i * np);
        out_cnt++;
        if (opt.force_call && out_cnt >= (int)positionMap.size()) stop = true;   // main.cpp:593 returns without a summary
      }
      B.n = 0;
      t_out += now_s() - t1;
      if (stuck) {   // (after the records: the reference had written them before exiting)
        fflush(vcf);
        std::rethrow_exception(stuck);
      }
    };

    std::vector<int> wpos(src.window()), rowOf(src.window());
    std::vector<uint8_t> wref(src.window());
    for (;;) {   // windows of Move2NextBaseEntry calls, merged serially, decoded and filled in parallel
      const int want = std::min(src.window(), B.cap - B.n);
      const double ti = now_s();
      const int got = src.nextSites(want, wpos.data(), wref.data());
      if (got > 0 && entries == 0) entries = src.maxPosition();
      for (int s = 0; s < got; s++) {
        rowOf[s] = -1;
        if (!opt.positionFile.empty()) {
          std::string key = label + ":" + std::to_string(wpos[s] + 1);
          if (!positionMap.count(key)) continue;
        }
        const int i = B.n++;
        B.pos[i] = wpos[s] + 1;
        B.ref[i] = wref[s];
        rowOf[s] = i;
      }
      src.fill(rowOf.data(), B.pl, B.dm);
      t_ingest += now_s() - ti;
      if (B.n == B.cap) flush();
      if (stop || src.ended()) break;
    }
    flush();
    if (stop) { fflush(vcf); return 0; }

    pm_counters C;
    eval.counters(&C);
    print_summary(label, entries, C, t0);
    fflush(vcf);
  }
  fclose(vcf);
  return 0;
}

int polymutt_main(int argc, char** argv, const ShardComm* comm, const EvaluatorFactory& make) {
  try {
    Options opt = parse_command_line(argc, argv);
    Pedigree ped;
    ped.load(opt.datFile, opt.pedFile);
    if (!opt.blocksOut.empty()) {   // --glf2blocks: GLF site stream -> dense indexed blocks, no engine
      if (opt.glfListFile.empty()) throw FatalError("--glf2blocks needs the GLF index file (-g)\n");
      if (comm && comm->world > 1) throw FatalError("--glf2blocks runs in one process\n");
      const long n = convert_glf_to_blocks(ped, opt.glfListFile, opt.blocksOut, default_io_threads(opt), opt.blockSites);
      printf("%ld sites written to %s\n", n, opt.blocksOut.c_str());
      return 0;
    }
    const pm_pedigree v = ped.view();
    const pm_params par = opt.params();
    std::unique_ptr<SiteEvaluator> ev = make(v, par, opt);
    return run_polymutt(opt, ped, *ev, comm);
  } catch (const FatalError& e) {
    printf("\nFATAL ERROR - \n%s\n\n", e.what());
    return 1;
  } catch (const BrentError& e) {
    printf("\nFATAL NUMERIC ERROR - %s\n\n", e.what());
    return 1;
  }
}

}  // namespace pmhost
