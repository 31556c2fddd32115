// blocks.h -- the dense indexed site-block format.
//
// A .pmb file holds the site stream PedigreeGLF produces from a pedigree's GLF files (the sections, and per
// site the position, refBase and every person's 10 PL bytes + depth|mapQ), already merged and densified,
// so a run reads blocks straight into the engine's input layout instead of inflating and merging
// n_person GLF files per site.  `polymutt --glf2blocks OUT.pmb` writes one; `--in_blocks FILE` reads it in
// place of `-g` and gives byte-identical VCFs.
//
// Layout (little-endian):
//   header   "PMB1" u32 n_person u32 block_sites u32 0
//   section  "SECT" i32 maxPosition u32 label_len label[label_len]
//     block  "BLK1" u32 n  i32 pos[n] (0-based)  u8 ref[n]  u8 pl[n][n_person][10]  u32 dm[n][n_person]
//   end      "SEND" u64 sites_in_section
//   index    "PIDX" u32 n_blocks, per block {u32 section, u32 n, i32 first_pos, i32 last_pos, u64 offset}
//   trailer  u64 index_offset "PMBE"
// The index gives random access to any block: a shard rank seeks to the first block of its position range
// (BlockSiteSource::seek) and skips the rest of a section after its range (skipSection), so no rank reads
// another rank's blocks.  The SEND marker of section s sits right after its last block, so its offset follows
// from that block's index entry (offset + 8 + n (4 + 1 + 14 n_person)).
#pragma once
#include <cstdint>
#include <cstdio>
#include <memory>
#include <string>
#include <vector>
#include "ingest.h"

namespace pmhost {

struct BlockIndexEntry {
  uint32_t section, n;
  int32_t first_pos, last_pos;
  uint64_t offset;
};

class BlockWriter {
 public:
  void open(const std::string& path, int n_person, int block_sites);
  void beginSection(const std::string& label, int maxPosition);
  void block(int n, const int* pos, const uint8_t* ref, const uint8_t* pl, const uint32_t* dm);
  void endSection();
  void close();   // writes the index and the trailer
  ~BlockWriter();

 private:
  void put(const void* p, size_t n);
  FILE* fh_ = nullptr;
  std::string path_;
  int np_ = 0, bs_ = 0;
  uint32_t section_ = 0;
  uint64_t sectionSites_ = 0, off_ = 0;
  bool inSection_ = false;
  std::vector<BlockIndexEntry> index_;
};

// Reads with pread at an explicit file offset: a block's header (positions, refBase) when nextSites reaches it,
// and the PL / depth rows straight into the caller's batch rows in fill() -- one read per run of consecutive rows,
// split into chunks read in parallel on the source's thread pool (no intermediate copy of the 14 B x n_person rows).
class BlockSiteSource : public SiteStream {
 public:
  void open(const std::string& path, int n_person, int threads = 1);
  ~BlockSiteSource();
  bool nextSection() override;
  const std::string& label() const override { return label_; }
  int maxPosition() const override { return maxPos_; }
  int window() const override { return 1024; }
  int nextSites(int maxSites, int* pos, uint8_t* ref) override;
  bool ended() const override { return ended_; }
  void fill(const int* rowOf, uint8_t* pl, uint32_t* dm) override;
  const std::vector<BlockIndexEntry>& index() const { return index_; }
  bool seek(int64_t lo, int64_t hi) override;   // by the block index (see SiteStream::seek)
  void skipSection() override;      // by the block index: straight to the section's end marker
  long blocksRead() const override { return blocksRead_; }

 private:
  bool loadBlock();   // false at the section end marker
  uint64_t sectionEnd() const;   // file offset of the current section's "SEND" (index required)
  void get(void* p, size_t n);   // n bytes at off_, advancing it
  void readAt(void* p, uint64_t off, size_t n) const;
  int fd_ = -1;
  uint64_t off_ = 0, size_ = 0;
  std::string path_;
  int np_ = 0;
  std::string label_;
  int maxPos_ = 0;
  bool inSection_ = false, ended_ = true;
  // the loaded block (its header, and the file offsets of its PL and depth rows) and the cursor into it; the last
  // nextSites call covered [lastBegin_, cur_)
  std::vector<int> pos_;
  std::vector<uint8_t> ref_;
  uint64_t plOff_ = 0, dmOff_ = 0;
  int n_ = 0, cur_ = 0, lastBegin_ = 0;
  std::vector<BlockIndexEntry> index_;
  int64_t section_ = -1;        // the current section's number (the index's section field)
  uint64_t sectionStart_ = 0;   // file offset of the current section's first block (or its "SEND")
  long blocksRead_ = 0;
  int64_t rangeHi_ = INT64_MAX;   // seek's hi: no block starting at or past it is read
  std::unique_ptr<TaskPool> pool_;
};

// Converts the GLF site stream of `ped` (index file glfIndexFile) into a .pmb file; returns the site count.
long convert_glf_to_blocks(const Pedigree& ped, const std::string& glfIndexFile, const std::string& out, int io_threads,
                           int block_sites);

}  // namespace pmhost
