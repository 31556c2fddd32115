// glf.h -- GLF v3 reader and multi-person site iterator.
//
// GlfFile restates glfHandler (core/glfHandler.cpp:22-317): 20-byte packed records
//   byte0 = refBase:4 (IUPAC bitmask, low nibble) | recordType:4 (0 end, 1 SNP, 2 indel)
//   u32 offset (delta position), u32 depth:24|minLLK:8, u8 mapQuality, u8 lk[10] (AA..TT phred)
// read through zlib (gzip or plain), with a large per-file decompression buffer instead of the
// reference's 1+19-byte gzread calls.
//
// SiteSource restates PedigreeGLF (src/PedigreeGLF.cpp:117-324): opens one GLF per person, walks
// sections in lock-step and emits, per site, the dense block row the engine consumes
// (pl[n_person][10], dm[n_person] = depth | mapQ<<24; zeros for absent persons/records).
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>
#include <zlib.h>
#include "pedigree.h"

namespace pmhost {

class GlfFile {
 public:
  ~GlfFile();
  bool open(const std::string& path);   // false if the file cannot be opened
  bool isOpen() const { return fh_ != nullptr || fd_ >= 0; }
  bool nextSection();
  bool nextEntry();
  bool nextBaseEntry();

  std::string label;
  int maxPosition = 0;
  int position = 0;
  bool endOfSection = true;
  // current record
  uint8_t refBase = 0, recordType = 0, mapQuality = 0;
  uint32_t depth = 0;
  uint8_t lk[10] = {0};

 private:
  size_t read(void* dst, size_t n);
  bool eof();
  gzFile fh_ = nullptr;
  int fd_ = -1;   // an uncompressed file: read() straight into buf_ (gzread's transparent mode copies once more)
  struct RawBuf {   // (a read buffer that is not zero-filled: 4000 persons' 64 KB buffers are written by read() first)
    std::unique_ptr<uint8_t[]> p;
    size_t n = 0;
    uint8_t* data() { return p.get(); }
    const uint8_t* data() const { return p.get(); }
    size_t size() const { return n; }
    uint8_t operator[](size_t i) const { return p[i]; }
    void resize(size_t k) { p.reset(new uint8_t[k]); n = k; }
  } buf_;
  size_t pos_ = 0, len_ = 0;
  bool zeof_ = false;
};

// readGLFannoFile (src/main.cpp:15-37): GLF index file -> {key: file name}
std::map<std::string, std::string> read_glf_index(const std::string& path);

class SiteSource {
 public:
  // Opens every person's GLF (key = (int)GLF_Index looked up in the index file).
  void open(const Pedigree& ped, const std::string& glfIndexFile);
  bool nextSection();                  // PedigreeGLF::Move2NextSection
  bool nextBaseEntry();                // PedigreeGLF::Move2NextBaseEntry
  const std::string& label() const { return files_[nonNull_].label; }
  int maxPosition() const { return files_[nonNull_].maxPosition; }
  int currentPos = 0;
  int refBase = 0;
  // Fill the dense block row of the current site.
  void fill(uint8_t* pl, uint32_t* dm) const;
  int nPerson() const { return (int)files_.size(); }

 private:
  std::vector<GlfFile> files_;
  std::vector<char> has_;   // handle != NULL
  std::vector<std::string> pids_;
  int nonNull_ = -1;
};

}  // namespace pmhost
