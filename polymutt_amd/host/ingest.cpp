// ingest.cpp -- see ingest.h.
#include "ingest.h"
#include <algorithm>
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
ParallelSiteSource::~ParallelSiteSource() { delete pool_; }

void ParallelSiteSource::open(const Pedigree& ped, const std::string& glfIndexFile, int threads, int window) {
  auto index = read_glf_index(glfIndexFile);
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
  pool_->run((n + 31) / 32, [&](int c) {
    for (int j = c * 32; j < std::min(n, (c + 1) * 32); j++)
      if (!path[j].empty()) ok[j] = files_[j].open(path[j]);
  });
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
  lastPos_.assign(window_, 0);
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
  std::vector<char> flag(files_.size(), 0);
  forChunks([&](int j) {
    flag[j] = files_[j].nextSection();
    Queue& Q = qs_[j];
    Q.head = -1; Q.tail = 0; Q.terminal = false;
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
    Q.tail -= Q.head;
    Q.head = 0;
  }
  const int target = std::max(Q.head, 0) + need;
  if ((int)Q.q.size() < target) Q.q.resize(target);
  GlfFile& g = files_[j];
  while (Q.tail < target && !Q.terminal) {   // glfHandler::NextBaseEntry, :195-204
    g.nextBaseEntry();
    GlfState& s = Q.q[Q.tail++];
    s.pos = g.position;
    s.dm = (g.depth & 0xFFFFFFu) | ((uint32_t)g.mapQuality << 24);
    std::memcpy(s.lk, g.lk, 10);
    s.ref = g.refBase;
    s.rt = g.recordType;
    if (g.recordType == 0) Q.terminal = true;
  }
}

int ParallelSiteSource::nextSites(int maxSites, int* pos, uint8_t* ref) {
  nLast_ = 0;
  if (ended_ || maxSites <= 0) return 0;
  maxSites = std::min(maxSites, window_);
  // a call advances a person at most once: maxSites + 1 states from the head cover the whole window
  forChunks([&](int j) { refill(j, maxSites + 1); });
  prevPos_ = currentPos_;
  for (int j : active_) headAtStart_[j] = qs_[j].head;
  const int maxPos = files_[nonNull_].maxPosition;
  const int na = (int)active_.size();
  int s = 0;
  for (; s < maxSites; s++) {   // PedigreeGLF::Move2NextBaseEntry, :282-324, one fused pass per call
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
  return s;
}

void ParallelSiteSource::fill(const int* rowOf, uint8_t* pl, uint32_t* dm) {
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
  forChunks([&](int j) {   // the merge's advance rule, replayed for this person
    int k = headAtStart_[j];
    int prev = prevPos_;
    for (int s = 0; s < n; s++) {
      if (state(j, k).pos == prev) k = next(j, k);
      const GlfState& st = state(j, k);
      const int cur = lastPos_[s];
      prev = cur;
      const int r = rowOf[s];
      if (r < 0) continue;
      uint8_t* P = pl + ((size_t)r * np + j) * 10;
      if (st.pos == cur) {
        std::memcpy(P, st.lk, 10);
        dm[(size_t)r * np + j] = st.dm;
      } else {
        std::memset(P, 0, 10);
        dm[(size_t)r * np + j] = 0;
      }
    }
  });
}

}  // namespace pmhost
