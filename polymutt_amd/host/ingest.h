// ingest.h -- parallel GLF ingest.
//
// ParallelSiteSource produces exactly the site stream of SiteSource (PedigreeGLF::Move2NextSection /
// Move2NextBaseEntry, src/PedigreeGLF.cpp:197-324), but splits the work the reference does serially per site:
//
//   1. decode  (parallel over persons): every person's GLF is inflated and parsed ahead into a queue of
//      GlfState -- the state glfHandler holds after each NextBaseEntry call (core/glfHandler.cpp:195-261).
//      A person's state sequence depends on its own file only, so the queues fill independently.
//   2. merge   (serial, integer only): Move2NextBaseEntry restated over the queue heads -- the end-of-section
//      check, the advance of the persons sitting at currentPos, and the min-position scan whose refBase is
//      taken from the first person holding the minimum.  One fused pass per site.
//   3. fill    (parallel over persons): each person replays the same advance rule over the merged positions
//      and writes its PL / depth|mapQ columns of the dense block rows.
//
// Memory: n_person x (window + 1) x 20 B of decoded states (82 MB for 4000 persons at the default window).
#pragma once
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include "glf.h"
#include "pedigree.h"

namespace pmhost {

// glfHandler's per-record state after a NextBaseEntry call.
struct GlfState {
  int32_t pos;
  uint32_t dm;       // depth (24 b) | mapQuality << 24
  uint8_t lk[10];
  uint8_t ref;       // translated refBase 0..4
  uint8_t rt;        // recordType (0 = end of section)
};

// Minimal fork-join pool: run(n, fn) calls fn(i) for i in [0, n) on the pool's threads and the caller.
class TaskPool {
 public:
  explicit TaskPool(int threads);
  ~TaskPool();
  void run(int n, const std::function<void(int)>& fn);
  int threads() const { return (int)workers_.size() + 1; }

 private:
  void work();
  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_ = 0, next_ = 0, active_ = 0;
  long gen_ = 0;
  bool stop_ = false;
};

// The driver's view of a site source: sections, then windows of sites and their dense block rows.
class SiteStream {
 public:
  virtual ~SiteStream() {}
  virtual bool nextSection() = 0;
  virtual const std::string& label() const = 0;
  virtual int maxPosition() const = 0;
  virtual int window() const = 0;
  // Up to maxSites (<= window) sites of the current section: pos[i] (0-based) and ref[i] (refBase).
  virtual int nextSites(int maxSites, int* pos, uint8_t* ref) = 0;
  virtual bool ended() const = 0;   // the current section has no more sites
  // Rows of the sites of the last nextSites call: site i -> row rowOf[i] (< 0: skipped).
  virtual void fill(const int* rowOf, uint8_t* pl, uint32_t* dm) = 0;
  // Random access (shards): restrict the current section to the blocks that overlap the 0-based positions
  // [lo, hi) -- skip to the first without reading what lies below lo, end the section before a block that
  // starts at or past hi.  Sites outside [lo, hi) may still come (the edge blocks); the caller drops them.
  // false: this source can only be read in order (GLF: an un-indexed, delta-coded gzip stream per person) and
  // the caller reads and drops the sites outside the range.
  virtual bool seek(int64_t lo, int64_t hi) { (void)lo; (void)hi; return false; }
  // Skip the rest of the current section without reading it (used after a shard's range ends).
  virtual void skipSection() {}
  virtual long blocksRead() const { return -1; }   // blocks loaded so far (-1: not a block source)
};

class ParallelSiteSource : public SiteStream {
 public:
  ParallelSiteSource() = default;
  ParallelSiteSource(const ParallelSiteSource&) = delete;
  ParallelSiteSource& operator=(const ParallelSiteSource&) = delete;
  ~ParallelSiteSource();
  // threads: decode/fill workers (the caller counts as one).  window: sites merged per nextSites call at most.
  void open(const Pedigree& ped, const std::string& glfIndexFile, int threads, int window = 4096);
  bool nextSection() override;   // PedigreeGLF::Move2NextSection (the files skip to their next section in parallel)
  const std::string& label() const override { return files_[nonNull_].label; }
  int maxPosition() const override { return files_[nonNull_].maxPosition; }
  int nPerson() const { return (int)files_.size(); }
  int window() const override { return window_; }
  bool ended() const override { return ended_; }

  // Advances up to maxSites (<= window) sites of the current section, as that many Move2NextBaseEntry calls
  // would: pos[i] (0-based currentPos) and ref[i] (refBase) of each site.  Returns the count; fewer than
  // maxSites means the section has ended.
  int nextSites(int maxSites, int* pos, uint8_t* ref) override;
  // Writes the block rows of the sites of the last nextSites call: site i goes to row rowOf[i] of pl
  // ([row][n_person][10]) and dm ([row][n_person]); rowOf[i] < 0 skips the site (--pos filtering).
  void fill(const int* rowOf, uint8_t* pl, uint32_t* dm) override;

 private:
  struct Queue {
    std::vector<GlfState> q;
    std::vector<int32_t> qp;   // q[k].pos, or INT32_MIN for an end-of-section record (fastMerge reads only this)
    int head = -1;          // -1: before the section's first call (the state at position 0)
    int tail = 0;
    bool terminal = false;  // q[tail - 1] is the end-of-section state, which repeats forever
  };
  void refill(int j, int need);
  void extend(int j, int target);
  void startAhead();
  void joinAhead();
  const GlfState& state(int j, int k) const { return k < 0 ? virtual_ : qs_[j].q[k]; }
  int next(int j, int k) const { return (k + 1 < qs_[j].tail) ? k + 1 : k; }
  template <class F> void forChunks(F f);

  std::vector<GlfFile> files_;
  std::vector<Queue> qs_;
  std::vector<int> active_;   // persons with a GLF handle (handle != NULL), ascending; active_[0] == nonNull_
  std::vector<char> has_;
  std::vector<std::string> pids_;
  int nonNull_ = -1;
  int window_ = 4096;
  TaskPool* pool_ = nullptr;
  GlfState virtual_{};
  int currentPos_ = 0;
  bool ended_ = false;
  // the last nextSites call: currentPos and queue heads before it, and the merged positions
  int prevPos_ = 0, nLast_ = 0;
  std::vector<int> headAtStart_, lastPos_, tailAtMerge_;
  TaskPool* dpool_ = nullptr;   // the decode-ahead's workers (startAhead)
  std::thread ahead_;
  double t_ahead_ = 0;
  double t_decode_ = 0, t_merge_ = 0, t_fill_ = 0;   // PM_TIMING: wall seconds per stage
  // the parallel merge of a run of calls (fastMerge; PM_SERIAL_MERGE=1 turns it off)
  int fastMerge(int maxSites, int maxPos, int* pos, uint8_t* ref);
  static constexpr int kFastRange = 1 << 14;   // positions scanned per parallel run at most
  struct Scratch { std::vector<uint32_t> stamp; std::vector<int64_t> who; };
  std::vector<Scratch> scratch_;
  std::vector<int> vend_;   // per active person: where fastMerge's scan of its valid prefix stopped
  uint32_t gen_ = 0;
  bool fast_ = true;
};

}  // namespace pmhost
