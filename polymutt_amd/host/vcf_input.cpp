// vcf_input.cpp -- see vcf_input.h.  Restates PedVCF::VarCallFromVCF (src/PedVCF.cpp:43-164) and the
// record handling of FamilyLikelihoodSeq_VCF (FillPenetrance :259-370, OutputVCF :412-521) with the
// libVcf field semantics they rely on (VCFRecord::getFormatIndex prefix match, VCFIndividual::get:
// a field is missing when absent or empty).  The likelihood work runs on the SiteEvaluator in vcf_mode.
#include "vcf_input.h"
#include <zlib.h>
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <vector>
#include <fcntl.h>
#include <unistd.h>
#include <chrono>
#include <memory>
#include <mutex>
#include <exception>
#include "ingest.h"
#include "vcf_fmt.h"

namespace pmhost {
namespace {

struct LineReader {   // plain or gzip text, lines of any length; offsets are in the uncompressed stream
  gzFile fh = nullptr;
  std::string path;
  std::vector<char> buf = std::vector<char>(1 << 20);
  ~LineReader() { if (fh) gzclose(fh); }
  bool open(const std::string& p) {
    path = p;
    fh = gzopen(p.c_str(), "rb");
    if (fh) gzbuffer(fh, 1 << 20);
    return fh != nullptr;
  }
  int64_t tell() const { return (int64_t)gztell(fh); }
  void seek(int64_t off) {   // plain files: a file seek; gzip: zlib re-inflates up to off (no parsing)
    if (gzseek(fh, (z_off_t)off, SEEK_SET) < 0) throw FatalError("VCF input " + path + ": seek failed\n");
  }
  int64_t size() {   // uncompressed bytes of the stream (gzip: one inflate pass), position kept
    const int64_t here = tell();
    int64_t n = 0;
    if (gzdirect(fh)) {
      FILE* f = fopen(path.c_str(), "rb");
      if (!f || fseek(f, 0, SEEK_END) != 0) throw FatalError("VCF input " + path + ": cannot size\n");
      n = (int64_t)ftell(f);
      fclose(f);
    } else {
      seek(0);
      int got;
      while ((got = gzread(fh, buf.data(), (unsigned)buf.size())) > 0) n += got;
      if (got < 0) throw FatalError("VCF input " + path + ": read error\n");
    }
    seek(here);
    return n;
  }
  bool next(std::string& line) {
    line.clear();
    for (;;) {
      if (!gzgets(fh, buf.data(), (int)buf.size())) return !line.empty();
      size_t n = strlen(buf.data());
      line.append(buf.data(), n);
      if (n && buf[n - 1] == '\n') {
        line.pop_back();
        if (!line.empty() && line.back() == '\r') line.pop_back();
        return true;
      }
    }
  }
};

// Whole lines of the stream, read in large blocks (one gzread per block instead of gzgets + append per line): a chunk's
// lines are pointers into the block, valid until the next chunk() call (which compacts and refills first).
// An uncompressed file is read with pread, in pieces of >= 4 MB on the pool's threads (the page-cache copy is the
// cost; one thread moved ~7 GB/s).
struct BlockReader {
  gzFile fh;
  int fd = -1;
  TaskPool* pool;
  std::vector<char> buf = std::vector<char>((size_t)64 << 20);
  size_t beg = 0, end = 0;
  int64_t base;   // uncompressed offset of buf[0]
  bool zeof = false;
  struct Line { const char* p; size_t n; int64_t off; };
  BlockReader(LineReader& lr, TaskPool* tp) : fh(lr.fh), pool(tp), base(lr.tell()) {
    if (const char* eb = getenv("PM_VCF_BLOCK")) buf.resize(std::max<size_t>(64, strtoull(eb, nullptr, 10)));   // (tests: refills)
    if (gzdirect(fh) && !getenv("PM_VCF_GZREAD")) {
      fd = ::open(lr.path.c_str(), O_RDONLY);
      if (fd >= 0) posix_fadvise(fd, 0, 0, POSIX_FADV_SEQUENTIAL);
    }
  }
  ~BlockReader() { if (fd >= 0) ::close(fd); }
  void fill() {   // buf[end, size) from the stream; zeof at its end
    if (fd < 0) {
      while (!zeof && end < buf.size()) {
        const int r = gzread(fh, buf.data() + end, (unsigned)std::min<size_t>(buf.size() - end, (size_t)1 << 30));
        if (r < 0) throw FatalError("VCF input: read error\n");
        if (r == 0) zeof = true;
        end += (size_t)r;
      }
      return;
    }
    const size_t want = buf.size() - end;
    const int64_t off0 = base + (int64_t)end;
    const int np = std::max(1, std::min(pool ? pool->threads() : 1, (int)(want >> 22)));
    std::vector<size_t> got(np, 0);
    std::vector<char> bad(np, 0);
    auto piece = [&](int i) {
      const size_t b = want * i / np, e = want * (i + 1) / np;
      size_t g = 0;
      while (b + g < e) {
        const ssize_t r = pread(fd, buf.data() + end + b + g, e - b - g, (off_t)(off0 + (int64_t)(b + g)));
        if (r < 0) { bad[i] = 1; break; }
        if (r == 0) break;
        g += (size_t)r;
      }
      got[i] = g;
    };
    if (np > 1) pool->run(np, piece);
    else piece(0);
    size_t total = 0;
    for (int i = 0; i < np; i++) {
      if (bad[i]) throw FatalError("VCF input: read error\n");
      total += got[i];
      if (got[i] < want * (i + 1) / np - want * i / np) { zeof = true; break; }   // (a regular file reads short only at its end)
    }
    end += total;
  }
  // Up to `max` whole lines ('\n' and a trailing '\r' removed); fewer when the block ends (the next call continues).
  void chunk(int max, std::vector<Line>& out) {
    out.clear();
    for (;;) {
      size_t at = beg;
      while ((int)out.size() < max && at < end) {
        const char* nl = (const char*)memchr(buf.data() + at, '\n', end - at);
        if (!nl) {
          if (!zeof) break;   // (a partial line: the next chunk, after the refill)
          nl = buf.data() + end;
        }
        size_t n = (size_t)(nl - (buf.data() + at));
        const size_t adv = n + (nl < buf.data() + end ? 1 : 0);
        if (n && buf[at + n - 1] == '\r') n--;
        out.push_back({buf.data() + at, n, base + (int64_t)at});
        at += adv;
      }
      beg = at;
      if (!out.empty() || zeof) return;
      // no whole line left: the partial one moved to the front (only now: compacting on every call moved most of the
      // block each time), then refilled; a line longer than the block grows it
      if (beg > 0) {
        memmove(buf.data(), buf.data() + beg, end - beg);
        base += (int64_t)beg;
        end -= beg;
        beg = 0;
      } else if (end == buf.size())
        buf.resize(buf.size() * 2);
      fill();
    }
  }
};

struct Span { int b = 0, e = 0; };

void split(const std::string& s, char sep, std::vector<Span>& out) {
  out.clear();
  int b = 0;
  const int n = (int)s.size();
  for (int i = 0; i <= n; i++)
    if (i == n || s[i] == sep) { out.push_back({b, i}); b = i + 1; }
}

// VCFRecord::getFormatIndex (libVcf/VCFRecord.h:283-308): first ':'-field that starts with `key`.
int format_index(const std::string& line, Span fmt, const char* key) {
  int b = fmt.b, idx = 0;
  const int e = fmt.e, kl = (int)strlen(key);
  while (b < e) {
    if (b + kl <= (int)line.size() && line.compare(b, kl, key) == 0) return idx;
    idx++;
    while (line[b++] != ':')
      if (b >= e) return -1;
  }
  return -1;
}

// VCFIndividual::get (libVcf/VCFIndividual.h:74-81): i-th ':' field; missing if absent or empty.
bool get_field(const std::string& line, Span col, int i, Span& out) {
  if (i < 0) return true;
  int b = col.b, k = 0;
  for (int p = col.b; p <= col.e; p++)
    if (p == col.e || line[p] == ':') {
      if (k == i) { out = {b, p}; return b == p; }
      k++;
      b = p + 1;
    }
  return true;
}

int allele2int(const std::string& a) {   // FamilyLikelihoodSeq_VCF::Allele2Int (:65-72)
  if (a == "A" || a == "a") return 1;
  if (a == "C" || a == "c") return 2;
  if (a == "G" || a == "g") return 3;
  if (a == "T" || a == "t") return 4;
  return 0;
}

// atoi(s) (the field runs to the next ':' / tab / end of line): plain digits without a call, anything else atoi itself
inline int atoi_fast(const char* s) {
  int v = 0;
  const char* q = s;
  while (*q >= '0' && *q <= '9' && q - s < 9) v = v * 10 + (*q++ - '0');
  if (q > s && !(*q >= '0' && *q <= '9')) return v;
  return atoi(s);
}

inline char* put_int_buf(char* w, int v) {   // fmt_int into a buffer
  char b[16];
  int n = 0;
  unsigned u = v < 0 ? 0u - (unsigned)v : (unsigned)v;
  do { b[n++] = char('0' + u % 10); u /= 10; } while (u);
  if (v < 0) *w++ = '-';
  while (n) *w++ = b[--n];
  return w;
}

int gi(int b1, int b2) { return b1 < b2 ? (b1 - 1) * (10 - b1) / 2 + (b2 - b1) : (b2 - 1) * (10 - b2) / 2 + (b1 - b2); }
bool is_ts(int a1, int a2) { return (a1 == 1 && a2 == 3) || (a1 == 2 && a2 == 4); }   // PedVCF::isTs (:25-28)

struct Pending {          // one record awaiting output, in file order
  std::string line;
  std::vector<Span> cols;
  bool computed = false;
  int slot = -1;
  int a1 = 0, a2 = 0;
  bool indel = false;
  int dp_idx = -1;        // DP's FORMAT index as it stood when the record was read: the reference writes each record at
                          // once (PedVCF.cpp:118-160), with DP looked up per record until found (:311-314)
  // classify_pre (parallel): the record's own facts; classify_apply (serial, in file order) the FORMAT state machine
  int bial = 0;           // 1 biallelic, 0 not
  int dp_c = -1, gl_c = -1, pl_c = -1;   // this record's FORMAT indices of DP / GL / PL
  void reset() {          // (keeps the line's and the columns' buffers: records are recycled, not reallocated)
    line.clear(); cols.clear();
    computed = false; slot = -1; a1 = a2 = 0; indel = false; dp_idx = -1; bial = 0; dp_c = gl_c = pl_c = -1;
  }
};

struct State {            // what FamilyLikelihoodSeq_VCF holds between records (stale output, :412-521)
  double qual = 0.0, min = 0.0;
  std::vector<pm_vcf_call> calls;    // per flattened person
  int a_ref = 0;                     // allele of the label convention (always allele1 in this path)
};


}  // namespace

// One record's FORMAT bookkeeping as the reference keeps it across records (FamilyLikelihoodSeq_VCF
// FillPenetrance :316-324): DP's index is looked up on every biallelic record until found; GL/PL once, on the first
// biallelic record.
struct FormatState {
  int GL_idx = -1, PL_idx = -1, DP_index = -1;
  bool frozen() const { return DP_index >= 0 && (GL_idx >= 0 || PL_idx >= 0); }
};

namespace {
void copy_file_into(const std::string& path, FILE* out) {
  FILE* in = fopen(path.c_str(), "rb");
  if (!in) throw FatalError("VCF shard merge: " + path + " is missing\n");
  std::vector<char> buf(1 << 20);
  size_t got;
  while ((got = fread(buf.data(), 1, buf.size(), in)) > 0) fwrite(buf.data(), 1, got, out);
  fclose(in);
}
int64_t pack_call(const pm_vcf_call& c) {
  return (int64_t)(uint8_t)c.best | ((int64_t)(uint8_t)c.gq << 8) | ((int64_t)(uint8_t)c.label << 16);
}
pm_vcf_call unpack_call(int64_t v) {
  pm_vcf_call c{(int8_t)(v & 0xFF), (int8_t)((v >> 8) & 0xFF), (int8_t)((v >> 16) & 0xFF), 0};
  return c;
}
double bits2d(int64_t v) { double d; memcpy(&d, &v, 8); return d; }
int64_t d2bits(double d) { int64_t v; memcpy(&v, &d, 8); return v; }
}  // namespace

// Sharded (comm->world > 1): rank R analyses the records whose lines start in its slice of the body's bytes
// (uncompressed offsets; gzip input is re-inflated up to the slice, never parsed) and writes their records to
// <out>.part<R>.  Cross-record state is handed over explicitly: the FORMAT indices come from a pre-scan of the
// records before the slice (normally just the first one), and the records a rank meets before its first
// record with data -- printed by the reference with the previous computed record's QUAL, AF and genotypes
// (PedVCF.cpp:113-122) -- are written after one all-gather that carries each rank's last computed state.
// Rank 0 then writes the header and concatenates the parts; the result is byte-identical to one process.
int run_polymutt_vcf(const Options& opt, const Pedigree& ped, SiteEvaluator& eval, const ShardComm* comm) {
  if (opt.vcfInFile == opt.vcfOutFile) throw FatalError("Input and output VCF files are the same!\n");
  if (opt.vcfOutFile.empty()) throw FatalError("vcfOutFile not provided for output!\n");
  const bool sharded = comm && (comm->world > 1 || comm->allgather);
  const int R = sharded ? comm->rank : 0, N = sharded ? comm->world : 1;
  LineReader in;
  if (!in.open(opt.vcfInFile)) throw FatalError("Cannot open VCF file " + opt.vcfInFile + "\n");

  const pm_pedigree pv = ped.view();
  const int np = pv.n_person;
  // pid -> flattened person (FamilyLikelihoodSeq_VCF::MapPID2Traverse :36-55, later families win)
  std::map<std::string, int> pid2person;
  for (int p = 0; p < np; p++) pid2person[ped.column_pid[p]] = p;

  std::string line;
  std::vector<Span> cols;
  std::vector<std::string> samples;
  while (in.next(line)) {
    if (line.compare(0, 2, "##") == 0) continue;
    if (line.compare(0, 1, "#") == 0) {
      split(line, '\t', cols);
      for (size_t i = 9; i < cols.size(); i++) samples.push_back(line.substr(cols[i].b, cols[i].e - cols[i].b));
      break;
    }
  }
  const int64_t body = in.tell();
  // included samples in VCF order (PedVCF.cpp:66-80); person index per VCF column (-1: not in the ped)
  std::vector<int> col_person(samples.size(), -1);
  std::vector<std::string> included;
  for (size_t i = 0; i < samples.size(); i++) {
    auto it = pid2person.find(samples[i]);
    if (it != pid2person.end()) { col_person[i] = it->second; included.push_back(samples[i]); }
  }

  std::vector<std::pair<int, int>> inc_cols;   // (VCF column, person) of the included samples, in VCF order
  for (size_t i = 0; i < samples.size(); i++)
    if (col_person[i] >= 0) inc_cols.push_back({(int)i, col_person[i]});

  auto write_header = [&](FILE* out) {
    std::string header = "#CHROM\tPOS\tID\tREF\tALT\tQUAL\tFILTER\tINFO\tFORMAT";
    for (auto& s : included) header += "\t" + s;
    fprintf(out, "##fileformat=VCFv4.1\n##Polymutt=%s\n", opt.cmd.c_str());
    fprintf(out, "%s",
            "##Note=VCF file modified by polymutt. Updated fileds include: QUAL, GT and GQ, AF and AC. NOTE: modification was "
            "applied only to biallelic variants\n"
            "##FILTER=<ID=LOWDP,Description=\"Low Depth filter when the average depth per sample is lessn than 1\">\n"
            "##INFO=<ID=DP,Number=1,Type=Integer,Description=\"Total Read Depth\">\n"
            "##INFO=<ID=AF,Number=A,Type=Float,Description=\"Alternative Allele Frequency\">\n"
            "##INFO=<ID=AC,Number=1,Type=Integer,Description=\"Alternative Allele Count\">\n"
            "##FORMAT=<ID=GT,Number=1,Type=String,Description=\"Genotype\">\n"
            "##FORMAT=<ID=GQ,Number=1,Type=Integer,Description=\"Genotype Quality\">\n"
            "##FORMAT=<ID=DP,Number=1,Type=Integer,Description=\"Read Depth\">\n"
            "##FORMAT=<ID=PL,Number=3,Type=Integer,Description=\"Phred-scaled Genotype Likelihoods\">\n"
            "##FORMAT=<ID=GL,Number=3,Type=Float,Description=\"Log10 Genotype Likelihoods\">\n");
    fprintf(out, "%s\n", header.c_str());
  };
  const std::string part = opt.vcfOutFile + ".part" + std::to_string(R), lead_in = part + ".lead", lead_out = part + ".leadvcf";
  FILE* out = fopen(sharded ? part.c_str() : opt.vcfOutFile.c_str(), "w");
  if (!out) throw FatalError("Open outpuf VCF file " + opt.vcfOutFile + " failed!\n");
  if (!sharded) write_header(out);

  // GetPolyPrior() once, before any SetNonAutosomeFlags (PedVCF.cpp:103): autosomal; GetPolyPrior_indel()
  // returns the same `prior` (NucFamGenotypeLikelihood.cpp:313).  PedVCF's own tstv_ratio is 2.0 (:7).
  double prior = 0;
  for (int i = 1; i <= 2 * pv.n_founders; i++) prior += 1.0 / i;
  prior *= opt.theta;
  const double tstv = 2.0, prior_ts = tstv / (tstv + 1), prior_tv = 0.5 / (tstv + 1);

  const int B = std::max(1, opt.batch);
  // Two batches: the main thread reads, classifies and parses records into one while the flusher thread runs the
  // engine on the other, formats its records and hands their text to the writer thread.  A batch's PL rows are in
  // page-locked memory where the evaluator offers it (an asynchronous, faster host-to-device copy); pend: its records
  // awaiting output, in file order; nb: its computed records.
  // The calls come back in their compact 4-B form (pm_engine_run_vcf), into page-locked memory too: widened into
  // pm_geno_call rows in pageable memory (0.45 GB per batch at 7000 samples) they were most of the engine stage.
  struct BatchBuf {
    SiteEvaluator& e;
    uint8_t* pl;
    pm_vcf_call* calls;   // (written by the engine before any read)
    std::vector<uint8_t> ref;
    std::vector<pm_site_result> res;
    std::vector<Pending*> pend;
    int nb = 0;
    BatchBuf(SiteEvaluator& ev, int b, int n)
        : e(ev), pl((uint8_t*)ev.host_alloc((size_t)b * n * 10)), calls((pm_vcf_call*)ev.host_alloc((size_t)b * n * sizeof(pm_vcf_call))),
          ref(b), res(b) {}
    ~BatchBuf() { e.host_free(pl); e.host_free(calls); }
  };
  BatchBuf bb0(eval, B, np), bb1(eval, B, np);
  BatchBuf* const bbs[2] = {&bb0, &bb1};
  if (!bb0.pl || !bb1.pl || !bb0.calls || !bb1.calls) throw FatalError("out of host memory\n");
  int cb = 0;   // the batch the main thread fills
  // records are recycled through a free list (their 10-100 KB line and column buffers are reused, not reallocated and
  // first-touched for every record); the flusher returns a batch's records to it
  std::vector<std::unique_ptr<Pending>> store;
  std::vector<Pending*> freel;
  std::mutex free_mu;
  auto take = [&]() -> Pending* {
    std::lock_guard<std::mutex> lk(free_mu);
    if (freel.empty()) { store.emplace_back(new Pending); return store.back().get(); }
    Pending* r = freel.back();
    freel.pop_back();
    return r;
  };
  int cur_chrom = -1, n_samples_with_data = 0, bad_allele = 0;
  FormatState fs;
  bool first = R == 0;   // FillPenetrance's first-record banner (:270-282): rank 0 owns the file's first record
  bool computed_any = false;
  int64_t n_lead = 0;
  FILE* lead = nullptr;   // sharded, R > 0: raw lines met before this rank's first record with data
  State st;
  st.calls.assign(np, pm_vcf_call{0, 0, PM_LBL_VCF_DIPLOID, 0});

  // The state a record is printed with: its own (a computed record) or the previous computed record's (a record
  // without data, PedVCF.cpp:113-122): QUAL, the AF minimiser and every person's call.
  struct RecState { double qual, min; const pm_vcf_call* calls; };
  auto fresh_state = [&](const Pending& r, const pm_site_result* Rs, const pm_vcf_call* C) {
    // mono/poly -> QUAL (PedVCF.cpp:136-152), with the reference's operator-precedence slip
    const double mono = Rs->varllk[0], poly = Rs->varllk[1];
    double llk_alt, llk_ref;
    if (!r.indel) {
      llk_alt = log10((prior * (is_ts(r.a1, r.a2) ? 1 : 0)) ? prior_ts : prior_tv) + poly;
      llk_ref = log10(1 - prior) + mono;
    } else {
      llk_alt = log10(prior) + poly;
      llk_ref = log10(1 - prior) + mono;
    }
    RecState S;
    if (llk_alt - llk_ref > 10) S.qual = 10.0 * (llk_alt - llk_ref);
    else {
      const double posterior = 1 / (1 + pow(10, llk_ref - llk_alt));
      S.qual = -10 * log10(1 - posterior);
    }
    S.min = Rs->af;
    S.calls = C;
    return S;
  };
  // OutputVCF (FamilyLikelihoodSeq_VCF.cpp:412-521): one record's text into `out` (no shared state: the records of a
  // batch are formatted in parallel).  One pass over each sample's column finds both its DP and its PL / GL subfield
  // (VCFIndividual::get: missing when absent or empty), then the text is written straight into `out`, sized to a bound
  // first (each sample adds at most 17 characters to the input bytes it copies)
  struct Fields { int db, de, pb, pe; };   // the DP and PL / GL subfields' spans (b < 0: missing)
  // GetBestGenoLabel_vcfv4 (NucFamGenotypeLikelihood.cpp:1590-1608)
  static const char* kDip[3] = {"0/0", "0/1", "1/1"};
  static const char* kHap[3] = {"0", "ERROR", "1"};
  auto format_record = [&](std::string& out, const Pending& r, const RecState& S) {
    thread_local std::vector<Fields> fv;
    const std::string& L = r.line;
    const char* lp = L.data();
    const int ia = r.dp_idx > 0 ? r.dp_idx : -1, ib = fs.PL_idx > 0 ? fs.PL_idx : fs.GL_idx, kmax = std::max(ia, ib);
    const size_t ns = inc_cols.size();
    fv.resize(ns);
    int AC = 0, totalDepth = 0;
    for (size_t s = 0; s < ns; s++) {
      const Span col = r.cols[9 + inc_cols[s].first];
      AC += S.calls[inc_cols[s].second].best;
      Fields F{-1, -1, -1, -1};
      int k = 0, b = col.b;
      for (int p = col.b; k <= kmax; p++) {
        const bool end = p == col.e;
        if (end || lp[p] == ':') {
          if (k == ia && p > b) { F.db = b; F.de = p; }
          if (k == ib && p > b) { F.pb = b; F.pe = p; }
          k++;
          b = p + 1;
          if (end) break;
        }
      }
      fv[s] = F;
      if (F.db >= 0) totalDepth += atoi_fast(lp + F.db);
    }
    out.resize(L.size() + 17 * ns + 1024);
    char* w = &out[0];
    auto put = [&](const char* p, size_t n) { memcpy(w, p, n); w += n; };
    auto fld = [&](int k) { put(lp + r.cols[k].b, (size_t)(r.cols[k].e - r.cols[k].b)); };
    for (int k = 0; k < 5; k++) {
      fld(k);
      if (k < 4) *w++ = '\t';
    }
    char head[512];
    auto putf = [&](int n) {   // (a text longer than head -- a QUAL of hundreds of digits -- grows the bound)
      if (n < (int)sizeof(head)) { put(head, (size_t)n); return; }
      const size_t at = (size_t)(w - &out[0]);
      out.resize(out.size() + (size_t)n);
      w = &out[0] + at;
    };
    int hn = snprintf(head, sizeof(head), "\t%.2f\t", S.qual);
    if (hn >= (int)sizeof(head)) { putf(hn); w += snprintf(w, (size_t)hn + 1, "\t%.2f\t", S.qual); } else putf(hn);
    fld(6);
    const char* fmt_s = fs.PL_idx > 0 ? "GT:GQ:DP:PL" : "GT:GQ:DP:GL";
    hn = snprintf(head, sizeof(head), "\tAF=%.2f;AC=%d;DP=%d\t%s", 1 - S.min, AC, totalDepth, fmt_s);
    if (hn >= (int)sizeof(head)) { putf(hn); w += snprintf(w, (size_t)hn + 1, "\tAF=%.2f;AC=%d;DP=%d\t%s", 1 - S.min, AC, totalDepth, fmt_s); }
    else putf(hn);
    for (size_t s = 0; s < ns; s++) {
      const pm_vcf_call& c = S.calls[inc_cols[s].second];
      const Fields& F = fv[s];
      const char* lab;
      if (c.label == PM_LBL_DOT) lab = ".";
      else if (c.gq <= 0) lab = "./.";
      else {
        const int bb = c.best < 0 || c.best > 2 ? 0 : c.best;
        lab = c.label == PM_LBL_VCF_HAPLOID ? kHap[bb] : kDip[bb];
      }
      *w++ = '\t';
      put(lab, strlen(lab));
      *w++ = ':';
      w = put_int_buf(w, (int)c.gq);
      *w++ = ':';
      if (F.db >= 0) put(lp + F.db, (size_t)(F.de - F.db));
      else *w++ = '.';
      *w++ = ':';
      if (F.pb >= 0) put(lp + F.pb, (size_t)(F.pe - F.pb));
      else *w++ = '.';
    }
    *w++ = '\n';
    out.resize((size_t)(w - &out[0]));
  };
  // the lead records of a shard, printed with the carried state, one at a time
  auto write_record = [&](FILE* fo, const Pending& r) {
    RecState S{st.qual, st.min, st.calls.data()};
    std::string t;
    format_record(t, r, S);
    fwrite(t.data(), 1, t.size(), fo);
  };

  TaskPool pool(std::max(1, std::min(16, opt.io_threads > 0 ? opt.io_threads : (int)std::thread::hardware_concurrency())));
  // PM_TIMING=1: wall seconds per stage on stderr at the end (read, split + classify, PL parse, engine, format, write)
  // (tm[6]: the whole record loop, wall)
  auto now = [] { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  double tm[8] = {0, 0, 0, 0, 0, 0, now(), 0};
  struct TimingOut {
    double* t;
    ~TimingOut() {
      if (getenv("PM_TIMING"))
        fprintf(stderr, "PM_TIMING vcf input: read %.3f s, classify %.3f s, parse %.3f s, engine %.3f s, format %.3f s, write %.3f s, "
                "loop %.3f s, flush wait %.3f s\n", t[0], t[1], t[2], t[3], t[4], t[5], t[6], t[7]);
    }
  } timing_out{tm};
  // (declared before the writer: on unwinding, ~Writer joins its thread before the texts it writes are destroyed)
  std::vector<std::string> texts[2];
  std::vector<RecState> states;
  // one writer thread: fwrite of a formatted batch, in order, overlapped with the work on the next batch
  struct Writer {
    std::thread th;
    bool fail = false;
    void start(FILE* f, const std::vector<std::string>* t, int n) {
      th = std::thread([this, f, t, n] {
        for (int k = 0; k < n && !fail; k++)
          if (fwrite((*t)[k].data(), 1, (*t)[k].size(), f) != (*t)[k].size()) fail = true;
      });
    }
    void wait() {
      if (th.joinable()) th.join();
      if (fail) throw FatalError("Write to the output VCF failed\n");
    }
    ~Writer() { if (th.joinable()) th.join(); }
  } writer;
  int tcur = 0;
  TaskPool fpool(pool.threads());   // (the flusher's: the main thread's pool parses the next batch meanwhile)
  auto process = [&](BatchBuf& bb) {   // the flusher's work on one batch, in batch order
    std::vector<Pending*>& pend = bb.pend;
    const pm_vcf_call* calls = bb.calls;
    int rows = 0;
    double t0 = now();
    // a Brent stuck at ITMAX (core/MathGold.cpp:98,175): the reference exits at that record, every earlier one written
    // (PedVCF.cpp:103-160 prints record by record): the batch's records before the stuck computed one go out, then the
    // error is raised
    std::exception_ptr stuck;
    size_t npend = pend.size();
    if (bb.nb > 0) {
      try {
        eval.run_vcf(bb.nb, np, bb.pl, bb.ref.data(), bb.res.data(), bb.calls, &rows);
      } catch (const BrentError& e) {
        stuck = std::current_exception();
        for (size_t k = 0; k < pend.size(); k++)
          if (pend[k]->computed && pend[k]->slot >= e.valid) { npend = k; break; }
      }
    }
    double t1 = now();
    tm[3] += t1 - t0;
    // the state each record prints with (sequential: a record without data takes the last computed one's)
    states.resize(npend);
    RecState cur{st.qual, st.min, st.calls.data()};
    for (size_t k = 0; k < npend; k++) {
      const Pending& r = *pend[k];
      if (r.computed) cur = fresh_state(r, &bb.res[r.slot], calls + (size_t)bb.res[r.slot].call_row * np);
      states[k] = cur;
    }
    std::vector<std::string>& T = texts[tcur];
    if (T.size() < npend) T.resize(npend);
    fpool.run((int)npend, [&](int k) { format_record(T[k], *pend[k], states[k]); });
    const double t2 = now();
    tm[4] += t2 - t1;
    // the batch's text goes out on the writer thread while the next batch is read, parsed and computed; the
    // previous batch's write finishes first (file order), then the buffers alternate
    writer.wait();
    tm[5] += now() - t2;   // (write: the time this thread waited for the writer)
    writer.start(out, &texts[tcur], (int)npend);
    tcur ^= 1;
    if (stuck) {
      writer.wait();
      fflush(out);
      std::rethrow_exception(stuck);
    }
    if (!pend.empty()) {   // the last state carries into the next batch
      st.qual = cur.qual; st.min = cur.min;
      if (cur.calls != st.calls.data()) std::copy(cur.calls, cur.calls + np, st.calls.begin());
    }
    {
      std::lock_guard<std::mutex> lk(free_mu);
      for (Pending* r : pend) freel.push_back(r);
    }
    pend.clear();
    bb.nb = 0;
  };
  std::thread flusher;
  std::exception_ptr ferr;
  auto drain = [&]() {   // the flusher's batch done (its errors raised here)
    const double tw = now();
    if (flusher.joinable()) flusher.join();
    tm[7] += now() - tw;
    if (ferr) std::rethrow_exception(ferr);
  };
  struct JoinAtExit {
    std::thread& t;
    ~JoinAtExit() { if (t.joinable()) t.join(); }
  } join_flusher{flusher};
  auto flush = [&]() {   // the filled batch to the flusher; the main thread goes on with the other (already drained)
    drain();
    BatchBuf* bb = bbs[cb];
    flusher = std::thread([&, bb] {
      try { process(*bb); } catch (...) { ferr = std::current_exception(); }
    });
    cb ^= 1;
  };

  // parses a record's columns and its biallelic / allele / FORMAT-index bookkeeping (:296-324); false: not output.
  // classify_pre: what depends on the record alone (any order, in parallel); classify_apply: the FORMAT bookkeeping
  // that carries from record to record, in file order
  auto classify_pre = [&](Pending& r) {
    split(r.line, '\t', r.cols);
    if (r.cols.size() < 9) return false;
    const std::string& L = r.line;
    const Span cr = r.cols[3], ca = r.cols[4];
    const std::string refS = L.substr(cr.b, cr.e - cr.b), altS = L.substr(ca.b, ca.e - ca.b);
    r.bial = refS != altS && altS.find(',') == std::string::npos;
    if (r.bial) {
      r.indel = refS.size() > 1 || altS.size() > 1;
      r.a1 = r.indel ? 1 : allele2int(refS);
      r.a2 = r.indel ? 2 : allele2int(altS);
      r.dp_c = format_index(L, r.cols[8], "DP");
      r.gl_c = format_index(L, r.cols[8], "GL");
      r.pl_c = format_index(L, r.cols[8], "PL");
    }
    return true;
  };
  auto classify_apply = [&](Pending& r) {
    if (r.cols.size() < 9) throw FatalError("Malformed VCF record (fewer than 9 columns)\n");
    const std::string& L = r.line;
    auto fld = [&](int k) { return L.substr(r.cols[k].b, r.cols[k].e - r.cols[k].b); };
    const bool biallelic = r.bial;
    if (biallelic) {
      if (fs.DP_index < 0) fs.DP_index = r.dp_c;
      r.dp_idx = fs.DP_index;
      if (fs.GL_idx < 0 && fs.PL_idx < 0) {
        fs.GL_idx = r.gl_c;
        fs.PL_idx = r.pl_c;
        if (fs.GL_idx < 0 && fs.PL_idx < 0) {
          fprintf(stderr, "NO GL or PL field was found. Please check the vcf file at chr:%s and position:%d", fld(0).c_str(),
                  atoi(fld(1).c_str()));
          exit(1);
        }
        if (included.empty()) throw FatalError("NO individual IDs match in the ped and vcf file!\n");
      }
      // non-ACGT single-base alleles index the genotype tables out of range in the reference (undefined
      // behaviour); a case-only REF/ALT difference gives a degenerate pair: both are skipped here
      if (r.a1 == 0 || r.a2 == 0 || r.a1 == r.a2) return -1;
    }
    return biallelic ? 1 : 0;
  };

  int64_t lo = body, hi = INT64_MAX;
  if (sharded) {
    // gzip input: one rank inflates the whole stream to learn its size and shares it (every rank doing so cost
    // O(file) inflation each); each rank then re-inflates only up to its own slice in seek()
    int64_t total;
    if (gzdirect(in.fh)) total = in.size();
    else {
      int64_t mine = R == 0 ? in.size() : 0;
      std::vector<int64_t> all(N);
      comm->allgather(&mine, 1, all.data());
      total = all[0];
    }
    lo = body + (total - body) * R / N;
    if (R < N - 1) hi = body + (total - body) * (R + 1) / N;
    if (R > 0) {
      // FORMAT indices as the records before the slice leave them (normally fixed by the first record)
      while (!fs.frozen() && in.tell() < lo && in.next(line)) {
        if (line.empty() || line[0] == '#') continue;
        Pending r;
        r.line.swap(line);
        classify_pre(r);
        classify_apply(r);
      }
      in.seek(lo - 1);   // the first line starting at or after lo: skip the rest of the line holding byte lo - 1
      in.next(line);
      lead = fopen(lead_in.c_str(), "w+b");
      if (!lead) throw FatalError("Open outpuf VCF file " + opt.vcfOutFile + " failed!\n");
    }
  }

  // Chunks of records: read and classified in order (the FORMAT bookkeeping carries from record to record), their
  // PL / GL fields parsed in parallel into per-record rows, then handled in order as the reference does.
  const int CH = 256;
  std::vector<Pending*> chunk(CH, nullptr);
  std::vector<int> kinds(CH), withdata(CH);
  std::vector<std::string> perr(CH);
  std::vector<uint8_t> rows((size_t)CH * np * 10);
  // FillPenetrance's per-sample loop (:338-382) for record k of the chunk: phred bytes of (geno11, geno12, geno22)
  auto parse_row = [&](int k) {
    const Pending& r = *chunk[k];
    const std::string& L = r.line;
    uint8_t* row = rows.data() + (size_t)k * np * 10;
    memset(row, 0, (size_t)np * 10);
    const int g0 = gi(r.a1, r.a1), g1 = gi(r.a1, r.a2), g2 = gi(r.a2, r.a2);
    const int gix[3] = {g0, g1, g2};
    const bool isPL = fs.PL_idx > 0;
    int wd = 0;
    perr[k].clear();
    Span f;
    for (size_t i = 0; i < samples.size(); i++) {
      const int p = col_person[i];
      if (p < 0) continue;
      if (get_field(L, r.cols[9 + i], fs.GL_idx > 0 ? fs.GL_idx : fs.PL_idx, f)) break;   // missing: the reference returns (:332-343)
      double v[3];
      int nv = 0, b = f.b;
      for (int q = f.b; q <= f.e; q++)
        if (q == f.e || L[q] == ',') {
          if (nv < 3) {
            // a plain decimal integer (the usual PL) without strtod; anything else through strtod as the reference's
            // String::AsDouble
            int d = 0, t = b;
            bool plain = isPL && q > b && q - b <= 9;
            for (; plain && t < q; t++) {
              const char ch = L[t];
              if (ch < '0' || ch > '9') plain = false;
              else d = d * 10 + (ch - '0');
            }
            v[nv] = plain ? (double)d : strtod(std::string(L, b, q - b).c_str(), nullptr);
          }
          nv++;
          b = q + 1;
        }
      if (nv != 3) {
        perr[k] = "GL or PL filed does not have 3 values separated by commas at: " + L.substr(r.cols[0].b, r.cols[0].e - r.cols[0].b) +
                  " " + L.substr(r.cols[1].b, r.cols[1].e - r.cols[1].b) + "!\n";
        break;
      }
      if (v[0] != 0.0 || v[1] != 0.0 || v[2] != 0.0) wd++;
      bool bad = false;
      for (int q = 0; q < 3; q++) {
        const int phred = (int)(isPL ? v[q] : -10 * v[q]);   // PL2LK(int(...)) (:361-363, :57-63)
        if (phred < 0) { perr[k] = "Phred-scaled likelihood " + std::to_string(phred) + " can not be negative\n"; bad = true; break; }
        row[(size_t)p * 10 + gix[q]] = (uint8_t)(phred > 255 ? 255 : phred);
      }
      if (bad) break;
    }
    withdata[k] = wd;
  };
  // a record's parsed row goes to its batch slot by a deferred copy, all of a chunk's (or a batch's) copies in parallel
  std::vector<std::pair<uint8_t*, int>> copies;   // (destination row, chunk record)
  auto do_copies = [&]() {
    const int nc2 = (int)copies.size();
    if (nc2 == 0) return;
    const int nt = std::min(nc2, 4 * pool.threads());
    pool.run(nt, [&](int t) {
      for (int q = (int)((int64_t)nc2 * t / nt); q < (int)((int64_t)nc2 * (t + 1) / nt); q++)
        memcpy(copies[q].first, rows.data() + (size_t)copies[q].second * np * 10, (size_t)np * 10);
    });
    copies.clear();
  };
  bool eof = false, stuck = false;
  BlockReader br(in, &pool);
  std::vector<BlockReader::Line> lines;
  std::vector<char> keep(CH);
  try {
  while (!eof) {
    // a chunk of lines from the block (in order), copied, split and classified in parallel, then the FORMAT
    // bookkeeping applied in file order
    double ta = now();
    br.chunk(CH, lines);
    double tb = now();
    tm[0] += tb - ta;
    if (lines.empty()) break;
    int nl = (int)lines.size();
    for (int k = 0; k < nl; k++)
      if (lines[k].off >= hi) { nl = k; eof = true; break; }   // (a shard's byte range ends before this line)
    for (int k = 0; k < nl; k++)
      if (!chunk[k]) chunk[k] = take();
    pool.run(nl, [&](int k) {
      const BlockReader::Line& l = lines[k];
      keep[k] = l.n > 0 && l.p[0] != '#';
      if (!keep[k]) return;
      Pending& r = *chunk[k];
      r.reset();
      r.line.assign(l.p, l.n);
      classify_pre(r);
    });
    int nc = 0;
    for (int k = 0; k < nl; k++) {
      if (!keep[k]) continue;
      if (nc != k) std::swap(chunk[nc], chunk[k]);
      Pending& r = *chunk[nc];
      if (first)   // FillPenetrance on the first record (:270-282) ...
        for (size_t i = 0; i < samples.size(); i++) {
          if (col_person[i] < 0) { printf("Sample ID \"%s\" not included in the analysis!\n", samples[i].c_str()); continue; }
          n_samples_with_data++;
        }
      kinds[nc] = classify_apply(r);
      if (first) {   // ... then VarCallFromVCF's banner (:117)
        printf("Total samples in both VCF and PED files: %d\n\n", n_samples_with_data);
        first = false;
      }
      nc++;
    }
    ta = now();
    tm[1] += ta - tb;
    pool.run(nc, [&](int k) { if (kinds[k] > 0) parse_row(k); });
    tm[2] += now() - ta;
    for (int k = 0; k < nc; k++) {
      const int kind = kinds[k];
      if (kind < 0) bad_allele++;
      if (kind <= 0) continue;   // OutputVCF returns at once for these records (:419)
      if (!perr[k].empty()) throw FatalError(perr[k]);
      Pending& r = *chunk[k];
      const std::string& L = r.line;
      // chromosome class of the record (PedVCF.cpp:121-124)
      const std::string chrom = L.substr(r.cols[0].b, r.cols[0].e - r.cols[0].b);
      const int cls = chrom == opt.chrX ? PM_CHR_X : chrom == opt.chrY ? PM_CHR_Y : chrom == opt.MT ? PM_CHR_MT : PM_CHR_AUTO;
      if (withdata[k] == 0) {   // written with the previous record's QUAL / AF / genotypes (:113)
        if (lead && !computed_any) {   // ... which an earlier rank computed: written after the exchange
          fprintf(lead, "%d\t%s\n", r.dp_idx, r.line.c_str());   // (with its DP index snapshot)
          n_lead++;
        } else {
          bbs[cb]->pend.push_back(chunk[k]);
          chunk[k] = nullptr;
        }
        continue;
      }
      computed_any = true;
      BatchBuf& bb = *bbs[cb];
      if (cls != cur_chrom) {
        do_copies();
        if (bb.nb > 0 || !bb.pend.empty()) flush();
        drain();   // (the engine's section changes: no batch of the old one in flight)
        eval.begin_section(cls);
        cur_chrom = cls;
      }
      BatchBuf& bc = *bbs[cb];
      copies.push_back({bc.pl + (size_t)bc.nb * np * 10, k});
      r.computed = true;
      r.slot = bc.nb;
      bc.ref[bc.nb] = (uint8_t)(r.a1 | (r.a2 << 4));
      bc.nb++;
      bc.pend.push_back(chunk[k]);
      chunk[k] = nullptr;
      if (bc.nb == B) {
        do_copies();
        flush();
      }
    }
    do_copies();
  }
  flush();
  drain();
  } catch (const BrentError&) {   // (process wrote the records before the stuck one; shards tell each other below)
    if (!sharded) throw;
    stuck = true;
  }
  {
    const double tw = now();
    writer.wait();
    tm[5] += now() - tw;
  }
  tm[6] = now() - tm[6];
  if (!sharded) {
    fclose(out);
    if (bad_allele) fprintf(stderr, "%d biallelic records with non-ACGT alleles were skipped\n", bad_allele);
    return 0;
  }

  // exchange: {computed any, QUAL, AF minimiser, skipped records, Brent stuck, the genotype calls} of each rank's last
  // computed record
  const int K = 5 + np;
  std::vector<int64_t> send(K), recv((size_t)N * K);
  send[0] = computed_any; send[1] = d2bits(st.qual); send[2] = d2bits(st.min); send[3] = bad_allele; send[4] = stuck;
  for (int p = 0; p < np; p++) send[5 + p] = pack_call(st.calls[p]);
  comm->allgather(send.data(), K, recv.data());
  int stuck_rank = -1;   // the first shard that met a stuck Brent: later shards' records come after it, never written
  for (int q = N - 1; q >= 0; q--)
    if (recv[(size_t)q * K + 4]) stuck_rank = q;
  fflush(out);
  fclose(out);
  if (lead) {   // this rank's leading no-data records, with the state of the nearest earlier rank that computed one
    State carried;
    carried.calls.assign(np, pm_vcf_call{0, 0, PM_LBL_VCF_DIPLOID, 0});
    for (int q = R - 1; q >= 0; q--) {
      const int64_t* v = recv.data() + (size_t)q * K;
      if (!v[0]) continue;
      carried.qual = bits2d(v[1]);
      carried.min = bits2d(v[2]);
      for (int p = 0; p < np; p++) carried.calls[p] = unpack_call(v[5 + p]);
      break;
    }
    std::swap(st, carried);
    FILE* lo_out = fopen(lead_out.c_str(), "wb");
    if (!lo_out) throw FatalError("Open outpuf VCF file " + opt.vcfOutFile + " failed!\n");
    LineReader lr;
    fflush(lead);
    fclose(lead);
    if (!lr.open(lead_in)) throw FatalError("VCF shard: " + lead_in + " is missing\n");
    for (int64_t k = 0; k < n_lead && lr.next(line); k++) {
      Pending r;
      const size_t tab = line.find('\t');
      r.dp_idx = atoi(line.c_str());
      r.line.assign(line, tab + 1, std::string::npos);
      split(r.line, '\t', r.cols);
      write_record(lo_out, r);
    }
    fclose(lo_out);
    remove(lead_in.c_str());
  }
  {   // every shard's files are complete before the lead concatenates them
    int64_t one = 1;
    std::vector<int64_t> all(N);
    comm->allgather(&one, 1, all.data());
  }
  if (R != 0) return stuck_rank >= 0 ? 1 : 0;   // (the lead prints the FATAL text once)
  FILE* fin = fopen(opt.vcfOutFile.c_str(), "w");
  if (!fin) throw FatalError("Open outpuf VCF file " + opt.vcfOutFile + " failed!\n");
  write_header(fin);
  int64_t bad = 0;
  for (int q = 0; q < N; q++) {
    const std::string pq = opt.vcfOutFile + ".part" + std::to_string(q);
    const bool keep_q = stuck_rank < 0 || q <= stuck_rank;
    if (q > 0) {
      if (keep_q) copy_file_into(pq + ".leadvcf", fin);
      remove((pq + ".leadvcf").c_str());
    }
    if (keep_q) copy_file_into(pq, fin);
    remove(pq.c_str());
    if (keep_q) bad += recv[(size_t)q * K + 3];
  }
  fclose(fin);
  if (bad) fprintf(stderr, "%lld biallelic records with non-ACGT alleles were skipped\n", (long long)bad);
  if (stuck_rank >= 0) throw BrentError();
  return 0;
}

}  // namespace pmhost
