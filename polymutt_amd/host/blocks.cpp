// blocks.cpp -- see blocks.h.
#include "blocks.h"
#include <algorithm>
#include <climits>
#include <cstring>
#include <cerrno>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

namespace pmhost {

BlockWriter::~BlockWriter() { if (fh_) fclose(fh_); }

void BlockWriter::put(const void* p, size_t n) {
  if (n && fwrite(p, 1, n, fh_) != n) throw FatalError("write to " + path_ + " failed\n");
  off_ += n;
}

void BlockWriter::open(const std::string& path, int n_person, int block_sites) {
  path_ = path;
  fh_ = fopen(path.c_str(), "wb");
  if (!fh_) throw FatalError("block file " + path + " can not be opened for output!\n");
  np_ = n_person; bs_ = block_sites;
  const uint32_t h[3] = {(uint32_t)n_person, (uint32_t)block_sites, 0};
  put("PMB1", 4);
  put(h, sizeof(h));
}

void BlockWriter::beginSection(const std::string& label, int maxPosition) {
  if (inSection_) endSection();
  const int32_t mp = maxPosition;
  const uint32_t len = (uint32_t)label.size();
  put("SECT", 4); put(&mp, 4); put(&len, 4); put(label.data(), len);
  inSection_ = true;
  sectionSites_ = 0;
}

void BlockWriter::block(int n, const int* pos, const uint8_t* ref, const uint8_t* pl, const uint32_t* dm) {
  if (n <= 0) return;
  index_.push_back({section_, (uint32_t)n, pos[0], pos[n - 1], off_});
  const uint32_t un = (uint32_t)n;
  put("BLK1", 4); put(&un, 4);
  put(pos, sizeof(int) * n);
  put(ref, n);
  put(pl, (size_t)n * np_ * 10);
  put(dm, (size_t)n * np_ * 4);
  sectionSites_ += n;
}

void BlockWriter::endSection() {
  if (!inSection_) return;
  put("SEND", 4); put(&sectionSites_, 8);
  inSection_ = false;
  section_++;
}

void BlockWriter::close() {
  if (!fh_) return;
  endSection();
  const uint64_t at = off_;
  const uint32_t nb = (uint32_t)index_.size();
  put("PIDX", 4); put(&nb, 4);
  for (const auto& e : index_) { put(&e.section, 4); put(&e.n, 4); put(&e.first_pos, 4); put(&e.last_pos, 4); put(&e.offset, 8); }
  put(&at, 8); put("PMBE", 4);
  if (fclose(fh_) != 0) throw FatalError("write to " + path_ + " failed\n");
  fh_ = nullptr;
}

// ---------------------------------------------------------------------------------------------
BlockSiteSource::~BlockSiteSource() { if (fd_ >= 0) ::close(fd_); }

void BlockSiteSource::readAt(void* p, uint64_t off, size_t n) const {
  char* d = (char*)p;
  while (n > 0) {
    const ssize_t got = ::pread(fd_, d, n, (off_t)off);
    if (got < 0 && errno == EINTR) continue;
    if (got <= 0) throw FatalError("block file " + path_ + " is truncated\n");
    d += got; off += (uint64_t)got; n -= (size_t)got;
  }
}

void BlockSiteSource::get(void* p, size_t n) {
  readAt(p, off_, n);
  off_ += n;
}

void BlockSiteSource::open(const std::string& path, int n_person, int threads) {
  path_ = path;
  fd_ = ::open(path.c_str(), O_RDONLY);
  if (fd_ < 0) throw FatalError("block file " + path + " can not be opened!\n");
  struct stat st;
  if (fstat(fd_, &st) != 0) throw FatalError("block file " + path + " can not be opened!\n");
  size_ = (uint64_t)st.st_size;
  posix_fadvise(fd_, 0, 0, POSIX_FADV_SEQUENTIAL);
  char magic[4];
  uint32_t h[3];
  get(magic, 4); get(h, sizeof(h));
  if (memcmp(magic, "PMB1", 4) != 0) throw FatalError(path + " is not a polymutt block file\n");
  if ((int)h[0] != n_person)
    throw FatalError(path + ": block file has " + std::to_string(h[0]) + " persons, the pedigree " + std::to_string(n_person) + "\n");
  np_ = n_person;
  // index (trailer: u64 index_offset "PMBE")
  if (size_ >= off_ + 12) {
    uint64_t at = 0;
    char end[4];
    readAt(&at, size_ - 12, 8); readAt(end, size_ - 4, 4);
    if (memcmp(end, "PMBE", 4) == 0 && at + 8 <= size_) {
      char tag[4];
      uint32_t nb = 0;
      readAt(tag, at, 4); readAt(&nb, at + 4, 4);
      if (memcmp(tag, "PIDX", 4) == 0) {
        index_.resize(nb);
        uint64_t o = at + 8;
        for (auto& e : index_) {
          readAt(&e.section, o, 4); readAt(&e.n, o + 4, 4); readAt(&e.first_pos, o + 8, 4); readAt(&e.last_pos, o + 12, 4);
          readAt(&e.offset, o + 16, 8);
          o += 24;
        }
      }
    }
  }
  if (threads > 1) pool_.reset(new TaskPool(threads));
}

bool BlockSiteSource::nextSection() {
  // skip what is left of the current section (the reference's NextSection skips the rest of the records)
  if (inSection_) skipSection();
  while (inSection_) loadBlock();
  char tag[4];
  if (off_ + 4 > size_) return false;
  get(tag, 4);
  if (memcmp(tag, "SECT", 4) != 0) return false;   // "PIDX": no more sections
  int32_t mp;
  uint32_t len;
  get(&mp, 4); get(&len, 4);
  label_.assign(len, '\0');
  if (len) get(&label_[0], len);
  maxPos_ = mp;
  inSection_ = true;
  ended_ = false;
  n_ = cur_ = lastBegin_ = 0;
  section_++;
  sectionStart_ = off_;
  rangeHi_ = INT64_MAX;
  return true;
}

uint64_t BlockSiteSource::sectionEnd() const {
  const BlockIndexEntry* last = nullptr;
  for (const auto& e : index_)
    if ((int64_t)e.section == section_) last = &e;
  if (!last) return sectionStart_;   // no blocks: the section's first record is its end marker
  return last->offset + 8 + (uint64_t)last->n * (4 + 1 + 14 * (uint64_t)np_);
}

bool BlockSiteSource::seek(int64_t lo, int64_t hi) {
  if (index_.empty() || !inSection_) return false;
  rangeHi_ = hi;
  uint64_t at = 0;
  bool found = false;
  for (const auto& e : index_)
    if ((int64_t)e.section == section_ && (int64_t)e.last_pos >= lo) { at = e.offset; found = true; break; }
  if (!found) at = sectionEnd();   // every block of the section lies below lo
  off_ = at;
  n_ = cur_ = lastBegin_ = 0;
  return true;
}

void BlockSiteSource::skipSection() {
  if (index_.empty() || !inSection_) return;   // no index: nextSection reads the rest in order
  off_ = sectionEnd();
  n_ = cur_ = lastBegin_ = 0;
  loadBlock();   // the "SEND" marker
  ended_ = true;
}

bool BlockSiteSource::loadBlock() {
  char tag[4];
  get(tag, 4);
  if (memcmp(tag, "SEND", 4) == 0) {
    uint64_t cnt;
    get(&cnt, 8);
    inSection_ = false;
    n_ = cur_ = lastBegin_ = 0;
    return false;
  }
  if (memcmp(tag, "BLK1", 4) != 0) throw FatalError(path_ + ": corrupt block\n");
  blocksRead_++;
  uint32_t n;
  get(&n, 4);
  n_ = (int)n;
  pos_.resize(n); ref_.resize(n);
  get(pos_.data(), 4 * (size_t)n);
  get(ref_.data(), n);
  plOff_ = off_;   // the rows are read in fill(), straight into the caller's buffers
  dmOff_ = plOff_ + (uint64_t)n * np_ * 10;
  off_ = dmOff_ + (uint64_t)n * np_ * 4;
  if (off_ > size_) throw FatalError("block file " + path_ + " is truncated\n");
  cur_ = lastBegin_ = 0;
  return true;
}

int BlockSiteSource::nextSites(int maxSites, int* pos, uint8_t* ref) {
  lastBegin_ = cur_;
  if (ended_) return 0;
  if (cur_ == n_) {
    if (rangeHi_ != INT64_MAX) {   // the next block (index entries are in file order) starts past the range
      const uint64_t at = off_;
      auto it = std::lower_bound(index_.begin(), index_.end(), at,
                                 [](const BlockIndexEntry& e, uint64_t o) { return e.offset < o; });
      if (it != index_.end() && it->offset == at && (int64_t)it->first_pos >= rangeHi_) { ended_ = true; return 0; }
    }
    if (!loadBlock()) { ended_ = true; lastBegin_ = cur_; return 0; }
  }
  const int k = std::min(maxSites, n_ - cur_);
  for (int i = 0; i < k; i++) { pos[i] = pos_[cur_ + i]; ref[i] = ref_[cur_ + i]; }
  cur_ += k;
  return k;
}

void BlockSiteSource::fill(const int* rowOf, uint8_t* pl, uint32_t* dm) {
  // runs of consecutive destination rows -> one PL and one depth read each, in chunks of <= 4 MB on the pool
  struct Piece { char* dst; uint64_t off; size_t len; };
  std::vector<Piece> pieces;
  const size_t rpl = (size_t)np_ * 10, rdm = (size_t)np_ * 4, chunk = (size_t)4 << 20;
  auto add = [&](char* dst, uint64_t off, size_t len) {
    for (size_t o = 0; o < len; o += chunk) pieces.push_back({dst + o, off + o, std::min(chunk, len - o)});
  };
  const int cnt = cur_ - lastBegin_;
  for (int i = 0; i < cnt;) {
    if (rowOf[i] < 0) { i++; continue; }
    int j = i + 1;
    while (j < cnt && rowOf[j] == rowOf[j - 1] + 1) j++;
    const int s = lastBegin_ + i, r = rowOf[i], m = j - i;
    add((char*)(pl + (size_t)r * rpl), plOff_ + (uint64_t)s * rpl, (size_t)m * rpl);
    add((char*)(dm + (size_t)r * np_), dmOff_ + (uint64_t)s * rdm, (size_t)m * rdm);
    i = j;
  }
  if (pool_ && pieces.size() > 1) {
    // a failed or short read on a worker is recorded and rethrown here, on the calling thread (TaskPool::run does not
    // carry exceptions: one escaping a worker would end the process without the "truncated" message)
    std::vector<std::string> err(pieces.size());
    pool_->run((int)pieces.size(), [&](int k) {
      try {
        readAt(pieces[k].dst, pieces[k].off, pieces[k].len);
      } catch (const std::exception& e) {
        err[k] = e.what();
      }
    });
    for (auto& e : err)
      if (!e.empty()) throw FatalError(e);
  } else {
    for (auto& p : pieces) readAt(p.dst, p.off, p.len);
  }
}

// ---------------------------------------------------------------------------------------------
long convert_glf_to_blocks(const Pedigree& ped, const std::string& glfIndexFile, const std::string& out, int io_threads,
                           int block_sites) {
  ParallelSiteSource src;
  src.open(ped, glfIndexFile, io_threads);
  const int np = (int)ped.column_pid.size();
  const int bs = std::max(1, block_sites);
  BlockWriter w;
  w.open(out, np, bs);
  std::vector<int> pos(bs), rowOf(src.window());
  std::vector<uint8_t> ref(bs), pl((size_t)bs * np * 10);
  std::vector<uint32_t> dm((size_t)bs * np);
  std::vector<int> wpos(src.window());
  std::vector<uint8_t> wref(src.window());
  long total = 0;
  while (src.nextSection()) {
    w.beginSection(src.label(), src.maxPosition());
    int n = 0;
    while (!src.ended()) {
      const int got = src.nextSites(std::min(src.window(), bs - n), wpos.data(), wref.data());
      for (int i = 0; i < got; i++) { rowOf[i] = n + i; pos[n + i] = wpos[i]; ref[n + i] = wref[i]; }
      src.fill(rowOf.data(), pl.data(), dm.data());
      n += got;
      if (n == bs || (src.ended() && n > 0)) { w.block(n, pos.data(), ref.data(), pl.data(), dm.data()); total += n; n = 0; }
    }
    w.endSection();
  }
  w.close();
  return total;
}

}  // namespace pmhost
