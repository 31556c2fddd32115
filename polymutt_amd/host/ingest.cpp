// ingest.cpp -- see ingest.h.
#include "ingest.h"
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace pmhost {

TaskPool::TaskPool(int threads) {
  for (int i = 1; i < threads; i++) workers_.emplace_back([this] { work(); });
}

TaskPool::~TaskPool() {
  {
    std::lock_guard<std::mutex> l(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : workers_) t.join();
}

void TaskPool::work() {
  long seen = 0;
  std::unique_lock<std::mutex> l(mu_);
  for (;;) {
    cv_.wait(l, [&] { return stop_ || gen_ != seen; });
    if (stop_) return;
    seen = gen_;
    active_++;
    while (next_ < n_) {
      const int i = next_++;
      l.unlock();
      (*fn_)(i);
      l.lock();
    }
    if (--active_ == 0) done_cv_.notify_all();
  }
}

void TaskPool::run(int n, const std::function<void(int)>& fn) {
  if (workers_.empty() || n <= 1) {
    for (int i = 0; i < n; i++) fn(i);
    return;
  }
  std::unique_lock<std::mutex> l(mu_);
  fn_ = &fn; n_ = n; next_ = 0; gen_++;
  cv_.notify_all();
  active_++;
  while (next_ < n_) {
    const int i = next_++;
    l.unlock();
    fn(i);
    l.lock();
  }
  active_--;
  done_cv_.wait(l, [&] { return active_ == 0; });
  fn_ = nullptr; n_ = 0;
}

// ---------------------------------------------------------------------------------------------
static double ing_now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

ParallelSiteSource::~ParallelSiteSource() {
  joinAhead();
  if (getenv("PM_TIMING"))
    fprintf(stderr, "PM_TIMING glf ingest: decode %.3f s, merge %.3f s, fill %.3f s (decode ahead %.3f s)\n", t_decode_, t_merge_,
            t_fill_, t_ahead_);
  delete dpool_;
  delete pool_;
}

// The decode-ahead of the next window (on its own pool, while the caller fills this window's rows): each person's
// queue grows at its tail only, within the capacity reserved at the section start, so the states fill() reads --
// those between the heads before and after the last merge -- are neither moved nor reallocated under it.
void ParallelSiteSource::startAhead() {
  if (!dpool_) return;
  ahead_ = std::thread([this] {
    const double t0 = ing_now();
    const int na = (int)active_.size();
    const int chunk = std::max(1, std::min(64, na / (4 * dpool_->threads()) + 1));
    dpool_->run((na + chunk - 1) / chunk, [&](int c) {
      for (int i = c * chunk; i < std::min(na, (c + 1) * chunk); i++) {
        const int j = active_[i];
        extend(j, std::max(qs_[j].head, 0) + window_ + 1);
      }
    });
    t_ahead_ += ing_now() - t0;
  });
}
void ParallelSiteSource::joinAhead() {
  if (ahead_.joinable()) ahead_.join();
}

void ParallelSiteSource::open(const Pedigree& ped, const std::string& glfIndexFile, int threads, int window) {
  const double to0 = ing_now();
  auto index = read_glf_index(glfIndexFile);
  const double to1 = ing_now();
  const int n = (int)ped.column_pid.size();
  files_ = std::vector<GlfFile>(n);
  qs_ = std::vector<Queue>(n);
  pids_ = ped.column_pid;
  has_.assign(n, 0);
  window_ = std::max(1, window);
  pool_ = new TaskPool(std::max(1, threads));
  // PedigreeGLF::SetPedGLF (src/PedigreeGLF.cpp:117-163): the file opens (inflate state + header) run in
  // parallel; warnings and the first open failure are then reported in person order, as the serial loop does
  std::vector<std::string> path(n), missing(n);
  for (int j = 0; j < n; j++) {
    const int idx = ped.column_glf[j];
    if (idx == 0) continue;
    const std::string key = std::to_string(idx);
    auto it = index.find(key);
    if (it == index.end()) missing[j] = key;
    else path[j] = it->second;
  }
  std::vector<char> ok(n, 0);
  const double to2 = ing_now();
  pool_->run((n + 31) / 32, [&](int c) {
    for (int j = c * 32; j < std::min(n, (c + 1) * 32); j++)
      if (!path[j].empty()) ok[j] = files_[j].open(path[j]);
  });
  if (getenv("PM_TIMING"))
    fprintf(stderr, "PM_TIMING glf open: index %.3f s, setup %.3f s, file opens %.3f s (%d threads)\n", to1 - to0, to2 - to1,
            ing_now() - to2, pool_->threads());
  for (size_t f = 0; f < ped.families.size(); f++) {
    int valid = 0;
    for (int j = ped.fam_start[f]; j < ped.fam_start[f + 1]; j++) {
      if (!missing[j].empty()) printf("\n\aWARNING - \nNo entry found for the glf with the key [%s]\n\n", missing[j].c_str());
      if (path[j].empty()) continue;
      if (!ok[j]) throw FatalError("GLF file " + path[j] + " can  not be opened!\n");
      has_[j] = 1;
      if (nonNull_ < 0) nonNull_ = j;
      valid++;
    }
    if (valid == 0) fprintf(stderr, "WARNING: No GLF files provided for family %s\n", ped.families[f].famid.c_str());
  }
  if (nonNull_ < 0) throw FatalError("No GLF file could be opened\n");
  for (int j = 0; j < n; j++)
    if (has_[j]) active_.push_back(j);
  headAtStart_.assign(n, -1);
  tailAtMerge_.assign(n, 0);
  if (threads > 1 && !getenv("PM_NO_DECODE_AHEAD")) {   // (PM_DECODE_THREADS: the decode-ahead pool's size, default threads / 2)
    const char* ed = getenv("PM_DECODE_THREADS");
    dpool_ = new TaskPool(std::max(1, ed ? atoi(ed) : threads / 2));
  }
  lastPos_.assign(window_, 0);
  fast_ = !getenv("PM_SERIAL_MERGE");
  virtual_.pos = 0;
  virtual_.rt = 0xFF;   // never inspected: the first call of a section skips the end check (currentPos == 0)
}

// Runs f(j) for every active person, in chunks over the pool.
template <class F>
void ParallelSiteSource::forChunks(F f) {
  const int na = (int)active_.size();
  const int chunk = std::max(1, std::min(64, na / (4 * pool_->threads()) + 1));
  const int nchunks = (na + chunk - 1) / chunk;
  pool_->run(nchunks, [&](int c) {
    const int e = std::min(na, (c + 1) * chunk);
    for (int i = c * chunk; i < e; i++) f(active_[i]);
  });
}

bool ParallelSiteSource::nextSection() {   // PedigreeGLF::Move2NextSection, :197-220
  joinAhead();
  std::vector<char> flag(files_.size(), 0);
  forChunks([&](int j) {
    flag[j] = files_[j].nextSection();
    Queue& Q = qs_[j];
    Q.head = -1; Q.tail = 0; Q.terminal = false;
    const size_t cap = 2 * (size_t)window_ + 4;   // (the decode-ahead never reallocates a queue)
    if (Q.q.size() < cap) { Q.q.resize(cap); Q.qp.resize(cap); }
  });
  const GlfFile& ref = files_[nonNull_];
  for (int j : active_) {   // checks in person order, as the serial loop makes them
    if (files_[j].maxPosition != ref.maxPosition || files_[j].label != ref.label) {
      char msg[1024];
      snprintf(msg, sizeof(msg),
               "GLF files are not compatible:\n\tFile of person %s has section %s with %d entries ...\n\tFile of person %s has section %s with %d entries ...\n",
               pids_[nonNull_].c_str(), ref.label.c_str(), ref.maxPosition, pids_[j].c_str(), files_[j].label.c_str(), files_[j].maxPosition);
      throw FatalError(msg);
    }
    if (!flag[j]) return false;
  }
  currentPos_ = 0;
  ended_ = false;
  nLast_ = 0;
  return true;
}

// Makes at least `need` states available from the queue head (fewer only at the section's end).
void ParallelSiteSource::refill(int j, int need) {
  Queue& Q = qs_[j];
  if (Q.head > 0) {   // drop consumed states
    std::memmove(Q.q.data(), Q.q.data() + Q.head, (size_t)(Q.tail - Q.head) * sizeof(GlfState));
    std::memmove(Q.qp.data(), Q.qp.data() + Q.head, (size_t)(Q.tail - Q.head) * sizeof(int32_t));
    Q.tail -= Q.head;
    Q.head = 0;
  }
  const int target = std::max(Q.head, 0) + need;
  if ((int)Q.q.size() < target) { Q.q.resize(target); Q.qp.resize(target); }
  extend(j, target);
}

// Decodes states at the queue's tail until it holds `target` (or the section's end record).
void ParallelSiteSource::extend(int j, int target) {
  Queue& Q = qs_[j];
  target = std::min(target, (int)Q.q.size());
  GlfFile& g = files_[j];
  while (Q.tail < target && !Q.terminal) {   // glfHandler::NextBaseEntry, :195-204
    g.nextBaseEntry();
    GlfState& s = Q.q[Q.tail++];
    s.pos = g.position;
    s.dm = (g.depth & 0xFFFFFFu) | ((uint32_t)g.mapQuality << 24);
    std::memcpy(s.lk, g.lk, 10);
    s.ref = g.refBase;
    s.rt = g.recordType;
    Q.qp[Q.tail - 1] = g.recordType == 0 ? INT32_MIN : g.position;   // (fastMerge's compact view)
    if (g.recordType == 0) Q.terminal = true;
  }
}

int ParallelSiteSource::nextSites(int maxSites, int* pos, uint8_t* ref) {
  nLast_ = 0;
  if (ended_ || maxSites <= 0) return 0;
  maxSites = std::min(maxSites, window_);
  // a call advances a person at most once: maxSites + 1 states from the head cover the whole window
  const double t0 = ing_now();
  joinAhead();   // (the previous window's fill is done: states before the heads may move now)
  forChunks([&](int j) { refill(j, maxSites + 1); });
  const double t1 = ing_now();
  t_decode_ += t1 - t0;
  prevPos_ = currentPos_;
  for (int j : active_) headAtStart_[j] = qs_[j].head;
  const int maxPos = files_[nonNull_].maxPosition;
  const int na = (int)active_.size();
  int s = 0;
  for (; s < maxSites; s++) {   // PedigreeGLF::Move2NextBaseEntry, :282-324, one fused pass per call
    if (fast_ && s < maxSites) {   // a run of calls merged in parallel where that is provably the same (fastMerge)
      const int got = fastMerge(maxSites - s, maxPos, pos + s, ref + s);
      if (got > 0) {
        for (int t = 0; t < got; t++) lastPos_[s + t] = pos[s + t];
        s += got - 1;
        continue;
      }
    }
    const int cp = currentPos_;
    int mn = 0;
    uint8_t rf = 0;
    bool end = false;
    for (int i = 0; i < na; i++) {
      const int j = active_[i];
      Queue& Q = qs_[j];
      const GlfState* st = Q.head < 0 ? &virtual_ : &Q.q[Q.head];
      // :284-292 (a person at its end-of-section record ends the section; independent of the advances
      // already made in this pass, which the next section's skip discards)
      if (cp > 0 && st->rt == 0) { end = true; break; }
      if (st->pos == cp) {   // :294-299
        Q.head = next(j, Q.head);
        st = &Q.q[Q.head];
      }
      if (i == 0 || st->pos < mn) { mn = st->pos; rf = st->ref; }   // :301-318, first person holding the min
    }
    if (end) { ended_ = true; break; }
    currentPos_ = mn;
    if (!(mn <= maxPos)) { ended_ = true; break; }   // :321
    pos[s] = mn;
    ref[s] = rf;
    lastPos_[s] = mn;
  }
  nLast_ = s;
  for (int j : active_) tailAtMerge_[j] = qs_[j].tail;
  t_merge_ += ing_now() - t1;
  if (!ended_) startAhead();   // the next window's states decode while fill() writes this one's rows
  return s;
}

// A run of Move2NextBaseEntry calls merged in parallel.  From a state where every person's head is a record (not
// the section-start placeholder, not an end-of-section record) and currentPos cp > 0, each person's upcoming heads
// are its next queued states (after the one at cp, which this call advances past).  While those are records with
// strictly increasing positions, the serial calls reduce to: the next currentPos is the smallest position > the
// previous one that any person holds, its refBase that of the first person (in person order) holding it, and a
// person's head after the run its first state past the run's second-to-last position.  lim = the least position up
// to which every person's states are known to be such records (exclusive); positions in (cp, lim) are collected per
// chunk of persons (first holder in the chunk), the chunks reduced in person order, and up to maxSites of them
// emitted.  Returns the number of calls made (0: the next call needs the serial pass -- a section start or end, a
// repeated position, a queue that ran short).  The emitted sites, refBases and heads are those of the serial pass.
int ParallelSiteSource::fastMerge(int maxSites, int maxPos, int* pos, uint8_t* ref) {
  const int cp = currentPos_;
  if (cp <= 0 || maxSites <= 0) return 0;
  const int na = (int)active_.size();
  const int nchunk = std::min(na, 2 * pool_->threads());
  if ((int)scratch_.size() < nchunk) scratch_.resize(nchunk);
  if ((int)vend_.size() < na) vend_.resize(na);
  std::vector<int> lim(nchunk, INT32_MAX);
  std::vector<char> bad(nchunk, 0);
  // one pass per person: its valid upcoming prefix (records, strictly increasing positions; vend_ = where it stops),
  // and, per chunk, the first holder (active index, state) of every position in (cp, cp + kFastRange)
  gen_++;
  pool_->run(nchunk, [&](int c) {
    Scratch& S = scratch_[c];
    if (S.stamp.empty()) { S.stamp.assign(kFastRange, 0); S.who.assign(kFastRange, 0); }
    const int i0 = (int)((long long)na * c / nchunk), i1 = (int)((long long)na * (c + 1) / nchunk);
    int l = INT32_MAX;
    for (int i = i0; i < i1; i++) {
      const Queue& Q = qs_[active_[i]];
      if (Q.head < 0) { bad[c] = 1; return; }
      const int32_t* qp = Q.qp.data();
      const int hp = qp[Q.head];   // (INT32_MIN: an end-of-section record)
      if (hp == INT32_MIN) { bad[c] = 1; return; }
      int k = hp == cp ? Q.head + 1 : Q.head, prev = cp;
      const int top = cp + kFastRange;
      // (INT32_MIN fails `> prev` too; positions past the range or the chunk's running limit need no stamp)
      for (; k < Q.tail && qp[k] > prev && qp[k] <= top && qp[k] < l; k++) {
        const int x = qp[k] - cp - 1;
        if (S.stamp[x] != gen_) { S.stamp[x] = gen_; S.who[x] = (int64_t)i << 32 | (uint32_t)k; }
        prev = qp[k];
      }
      vend_[i] = k;
      if (k < Q.tail && qp[k] > prev) continue;   // (stopped at the range or the running limit, not at a bad record)
      if (prev == cp) { bad[c] = 1; return; }     // no usable upcoming record
      l = prev;   // the last record of the valid prefix (a repeat, an end record or the queue's end follows)
    }
    lim[c] = l;
  });
  int H = INT32_MAX;
  for (int c = 0; c < nchunk; c++) {
    if (bad[c]) return 0;
    H = std::min(H, lim[c]);
  }
  H = std::min(H, maxPos + 1);   // (a position past maxPosition ends the section: the serial pass)
  if (H - cp - 1 > kFastRange) H = cp + 1 + kFastRange;
  const int R = H - cp - 1;   // positions cp + 1 .. H - 1: every person's states there are stamped
  if (R <= 0) return 0;
  // reduce in person order (chunks ascending), emit ascending
  int m = 0;
  for (int x = 0; x < R && m < maxSites; x++)
    for (int c = 0; c < nchunk; c++)
      if (scratch_[c].stamp[x] == gen_) {
        const int64_t w = scratch_[c].who[x];
        const int j = active_[(int)(w >> 32)];
        pos[m] = cp + 1 + x;
        ref[m] = qs_[j].q[(uint32_t)w].ref;
        m++;
        break;
      }
  if (m == 0) return 0;
  // heads: each person's first state past the second-to-last emitted position (cp when one site was emitted), found
  // by binary search in its valid prefix (strictly increasing; the head sought lies in it, at or below H)
  const int before = m >= 2 ? pos[m - 2] : cp;
  pool_->run(nchunk, [&](int c) {
    const int i0 = (int)((long long)na * c / nchunk), i1 = (int)((long long)na * (c + 1) / nchunk);
    for (int i = i0; i < i1; i++) {
      Queue& Q = qs_[active_[i]];
      if (Q.qp[Q.head] > before) continue;
      const int32_t* b = Q.qp.data() + Q.head + 1;
      Q.head = (int)(std::upper_bound(b, (const int32_t*)Q.qp.data() + vend_[i], before) - Q.qp.data());
    }
  });
  currentPos_ = pos[m - 1];
  return m;
}

void ParallelSiteSource::fill(const int* rowOf, uint8_t* pl, uint32_t* dm) {
  const double t0 = ing_now();
  struct Acc { double& t; double t0; ~Acc() { t += ing_now() - t0; } } acc{t_fill_, t0};
  const size_t np = files_.size();
  const int n = nLast_;
  for (size_t j = 0; j < np; j++) {   // persons without a handle: zero columns (SiteSource::fill)
    if (has_[j]) continue;
    for (int s = 0; s < n; s++) {
      if (rowOf[s] < 0) continue;
      std::memset(pl + ((size_t)rowOf[s] * np + j) * 10, 0, 10);
      dm[(size_t)rowOf[s] * np + j] = 0;
    }
  }
  // the merge's advance rule replayed per person, for a chunk of up to 64 persons at a time with the sites outer, so each
  // site row receives the chunk's contiguous 640 PL bytes (columns of a row) rather than one 10-byte piece per row
  const int na = (int)active_.size();
  static const int kFillChunk = [] {   // persons per chunk (PM_FILL_CHUNK, 1-64): the queues a thread streams at once
    const char* e = getenv("PM_FILL_CHUNK");
    return e ? std::max(1, std::min(64, atoi(e))) : 64;
  }();
  const int FC = kFillChunk;
  const int nch = (na + FC - 1) / FC;
  pool_->run(nch, [&](int c) {
    const int i0 = c * FC, i1 = std::min(na, i0 + FC), m = i1 - i0;
    // per person of the chunk: its column, queue base and last index (the section-start placeholder only
    // as the first head: handled by state() before the site loop)
    int k[64], col[64], last[64];
    const GlfState* qb[64];
    int prev = prevPos_;
    for (int i = 0; i < m; i++) {
      const int j = active_[i0 + i];
      col[i] = j;
      qb[i] = qs_[j].q.data();
      last[i] = tailAtMerge_[j] - 1;   // (the tail as the merge saw it: the decode-ahead may be extending it)
      k[i] = headAtStart_[j];
    }
    for (int s = 0; s < n; s++) {
      const int cur = lastPos_[s];
      const int r = rowOf[s];
      uint8_t* prow = r >= 0 ? pl + (size_t)r * np * 10 : nullptr;
      uint32_t* drow = r >= 0 ? dm + (size_t)r * np : nullptr;
      for (int i = 0; i < m; i++) {
        int kk = k[i];
        const GlfState* st = kk < 0 ? &virtual_ : qb[i] + kk;
        if (st->pos == prev) {   // next(): the queue's last state repeats (the end-of-section record)
          kk = kk < last[i] ? kk + 1 : kk;
          k[i] = kk;
          st = kk < 0 ? &virtual_ : qb[i] + kk;
        }
        if (!prow) continue;
        uint8_t* P = prow + (size_t)col[i] * 10;
        if (st->pos == cur) {
          std::memcpy(P, st->lk, 10);
          drow[col[i]] = st->dm;
        } else {
          std::memset(P, 0, 10);
          drow[col[i]] = 0;
        }
      }
      prev = cur;
    }
  });
}

}  // namespace pmhost
