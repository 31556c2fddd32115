// glf.cpp -- see glf.h.
#include "glf.h"
#include <fcntl.h>
#include <unistd.h>
#include <cstdio>
#include <cstring>

namespace pmhost {

static const uint8_t kTranslateBase[16] = {0, 1, 2, 0, 3, 0, 0, 0, 4, 0, 0, 0, 0, 0, 0, 0};   // glfHandler.cpp:4

GlfFile::~GlfFile() {
  if (fh_) gzclose(fh_);
  if (fd_ >= 0) ::close(fd_);
}

bool GlfFile::open(const std::string& path) {
  // gzip (magic 1f 8b) through zlib; anything else is read as it is, as zlib's transparent mode would (gzdirect),
  // with plain read() calls -- decided from two bytes, so opening a plain file reads nothing more
  const int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) return false;
  uint8_t mg[2] = {0, 0};
  const bool gz = ::pread(fd, mg, 2, 0) == 2 && mg[0] == 0x1f && mg[1] == 0x8b;
  if (gz) {
    ::close(fd);
    fh_ = gzopen(path.c_str(), "rb");
    if (!fh_) return false;
    gzbuffer(fh_, 1 << 16);
  } else {
    posix_fadvise(fd, 0, 0, POSIX_FADV_SEQUENTIAL);
    fd_ = fd;
  }
  buf_.resize(1 << 16);
  pos_ = len_ = 0;
  zeof_ = false;
  // glfHandler::ReadHeader (:87-134): "GLF\3", u32 header length, header text
  uint8_t magic[4];
  uint32_t hlen = 0;
  if (read(magic, 4) != 4 || magic[0] != 'G' || magic[1] != 'L' || magic[2] != 'F' || magic[3] != 3 ||
      read(&hlen, 4) != 4 || hlen > 1024 * 1024) {
    if (fh_) gzclose(fh_);
    fh_ = nullptr;
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
    return false;
  }
  std::vector<char> h(hlen);
  if (hlen && read(h.data(), hlen) != hlen) {
    if (fh_) gzclose(fh_);
    fh_ = nullptr;
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
    return false;
  }
  endOfSection = true;
  return true;
}

size_t GlfFile::read(void* dst, size_t n) {
  uint8_t* d = (uint8_t*)dst;
  size_t got = 0;
  while (got < n) {
    if (pos_ == len_) {
      if (zeof_) break;
      const int r = fd_ >= 0 ? (int)::read(fd_, buf_.data(), buf_.size()) : gzread(fh_, buf_.data(), (unsigned)buf_.size());
      if (r <= 0) { zeof_ = true; break; }
      len_ = (size_t)r; pos_ = 0;
    }
    size_t k = std::min(n - got, len_ - pos_);
    memcpy(d + got, buf_.data() + pos_, k);
    pos_ += k; got += k;
  }
  return got;
}

// ifeof(): true once a read has hit the end of the stream
bool GlfFile::eof() { return zeof_ && pos_ == len_; }

// glfHandler::NextSection (:163-193)
bool GlfFile::nextSection() {
  while (!endOfSection && !eof()) nextEntry();
  endOfSection = false;
  position = 0;
  int32_t labelLength = 0;
  if (read(&labelLength, 4) == 4) {
    std::vector<char> lab((size_t)(labelLength > 0 ? labelLength : 0) + 1, 0);
    if (labelLength > 0) read(lab.data(), (size_t)labelLength);
    label.assign(lab.data(), strnlen(lab.data(), lab.size()));
    maxPosition = 0;
    read(&maxPosition, 4);
    return maxPosition > 0 && !eof();
  }
  return false;
}

// glfHandler::NextEntry (:206-261)
bool GlfFile::nextEntry() {
  uint8_t b0;
  if (!endOfSection && len_ - pos_ >= 20 && (buf_[pos_] >> 4) == 1) {   // a whole record in the buffer: parse in place
    const uint8_t* r = (const uint8_t*)buf_.data() + pos_;
    uint32_t off, dm;
    memcpy(&off, r + 1, 4); memcpy(&dm, r + 5, 4);
    refBase = kTranslateBase[r[0] & 0xF];
    recordType = 1;
    depth = dm & 0xFFFFFF;
    mapQuality = r[9];
    memcpy(lk, r + 10, 10);
    position += (int)off;
    pos_ += 20;
    return true;
  }
  if (endOfSection || read(&b0, 1) != 1) {
    endOfSection = true; recordType = 0; position = maxPosition + 1;
    return false;
  }
  refBase = b0 & 0xF;
  recordType = b0 >> 4;
  switch (recordType) {
    case 0:
      endOfSection = true; position = maxPosition + 1;
      return true;
    case 1: {
      uint8_t r[19];
      if (read(r, 19) == 19) {
        uint32_t off, dm;
        memcpy(&off, r, 4); memcpy(&dm, r + 4, 4);
        refBase = kTranslateBase[refBase];
        depth = dm & 0xFFFFFF;
        mapQuality = r[8];
        memcpy(lk, r + 9, 10);
        position += (int)off;
        return true;
      }
      recordType = 0; position = maxPosition + 1;
      return false;
    }
    case 2: {
      uint8_t r[16];
      if (read(r, 16) == 16) {
        uint32_t off, dm;
        int16_t l0, l1;
        memcpy(&off, r, 4); memcpy(&dm, r + 4, 4);
        refBase = kTranslateBase[refBase];
        depth = dm & 0xFFFFFF;
        mapQuality = r[8];
        memcpy(lk, r + 9, 7);   // union with glfIndel: lk[0..2] likelihoods, lk[3..6] lengths
        memcpy(&l0, r + 12, 2); memcpy(&l1, r + 14, 2);
        position += (int)off;
        std::vector<char> skip((size_t)std::abs(l0) + (size_t)std::abs(l1) + 1);
        if (read(skip.data(), (size_t)std::abs(l0)) != (size_t)std::abs(l0)) { recordType = 0; position = maxPosition + 1; return false; }
        if (read(skip.data(), (size_t)std::abs(l1)) != (size_t)std::abs(l1)) { recordType = 0; position = maxPosition + 1; return false; }
        return true;
      }
      recordType = 0; position = maxPosition + 1;
      return false;
    }
  }
  return false;
}

bool GlfFile::nextBaseEntry() {   // :195-204
  bool r;
  do { r = nextEntry(); } while (r && recordType == 2);
  return r;
}

// ---------------------------------------------------------------------------------------------
std::map<std::string, std::string> read_glf_index(const std::string& path) {
  // readGLFannoFile, src/main.cpp:15-37: "key filename" per line, lines with <2 tokens skipped
  std::map<std::string, std::string> m;
  gzFile fh = gzopen(path.c_str(), "rb");
  if (!fh) throw FatalError(path + " open failed\n");
  std::string line;
  int c;
  auto flush = [&]() {
    std::vector<std::string> t;
    size_t i = 0;
    while (i < line.size()) {
      while (i < line.size() && isspace((unsigned char)line[i])) i++;
      size_t j = i;
      while (j < line.size() && !isspace((unsigned char)line[j])) j++;
      if (j > i) t.push_back(line.substr(i, j - i));
      i = j;
    }
    if (t.size() >= 2 && !m.count(t[0])) m[t[0]] = t[1];
    line.clear();
  };
  while ((c = gzgetc(fh)) != -1) {
    if (c == '\n') flush(); else line.push_back((char)c);
  }
  flush();
  gzclose(fh);
  return m;
}

void SiteSource::open(const Pedigree& ped, const std::string& glfIndexFile) {
  auto index = read_glf_index(glfIndexFile);
  const int n = (int)ped.column_pid.size();
  files_ = std::vector<GlfFile>(n);
  has_.assign(n, 0);
  pids_ = ped.column_pid;
  for (size_t f = 0; f < ped.families.size(); f++) {   // PedigreeGLF::SetPedGLF, src/PedigreeGLF.cpp:117-163
    int valid = 0;
    for (int j = ped.fam_start[f]; j < ped.fam_start[f + 1]; j++) {
      int idx = ped.column_glf[j];
      if (idx == 0) continue;
      std::string key = std::to_string(idx);
      auto it = index.find(key);
      if (it == index.end()) {
        printf("\n\aWARNING - \nNo entry found for the glf with the key [%s]\n\n", key.c_str());
        continue;
      }
      if (!files_[j].open(it->second)) throw FatalError("GLF file " + it->second + " can  not be opened!\n");
      has_[j] = 1;
      if (nonNull_ < 0) nonNull_ = j;
      valid++;
    }
    if (valid == 0) fprintf(stderr, "WARNING: No GLF files provided for family %s\n", ped.families[f].famid.c_str());
  }
  if (nonNull_ < 0) throw FatalError("No GLF file could be opened\n");
}

bool SiteSource::nextSection() {   // PedigreeGLF::Move2NextSection, :197-220
  bool flag = false;
  GlfFile& ref = files_[nonNull_];
  for (size_t j = 0; j < files_.size(); j++) {
    if (!has_[j]) continue;
    flag = files_[j].nextSection();
    if (files_[j].maxPosition != ref.maxPosition || files_[j].label != ref.label) {
      char msg[1024];
      snprintf(msg, sizeof(msg),
               "GLF files are not compatible:\n\tFile of person %s has section %s with %d entries ...\n\tFile of person %s has section %s with %d entries ...\n",
               pids_[nonNull_].c_str(), ref.label.c_str(), ref.maxPosition, pids_[j].c_str(), files_[j].label.c_str(), files_[j].maxPosition);
      throw FatalError(msg);
    }
    if (!flag) return flag;
  }
  currentPos = 0;
  return flag;
}

bool SiteSource::nextBaseEntry() {   // PedigreeGLF::Move2NextBaseEntry, :282-324
  if (currentPos > 0)
    for (size_t j = 0; j < files_.size(); j++)
      if (has_[j] && files_[j].recordType == 0) return false;
  for (size_t j = 0; j < files_.size(); j++)
    if (has_[j] && files_[j].position == currentPos) files_[j].nextBaseEntry();
  const GlfFile& nn = files_[nonNull_];
  currentPos = nn.position;
  refBase = nn.refBase;
  for (size_t j = 0; j < files_.size(); j++)
    if (has_[j] && files_[j].position < currentPos) { currentPos = files_[j].position; refBase = files_[j].refBase; }
  return currentPos <= nn.maxPosition;
}

void SiteSource::fill(uint8_t* pl, uint32_t* dm) const {
  for (size_t j = 0; j < files_.size(); j++) {
    const GlfFile& g = files_[j];
    if (has_[j] && g.position == currentPos) {
      memcpy(pl + j * 10, g.lk, 10);
      dm[j] = (g.depth & 0xFFFFFFu) | ((uint32_t)g.mapQuality << 24);
    } else {
      memset(pl + j * 10, 0, 10);
      dm[j] = 0;
    }
  }
}

}  // namespace pmhost
