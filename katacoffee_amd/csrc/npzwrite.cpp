// .npz training-data files in the reference's layout (TrainingWriteBuffers::
// writeToZipFile trainingwrite.cpp:566-587, NumpyBuffer numpywrite.cpp:100-175):
// a zip archive with five members named binaryInputNCHWPacked, globalInputNC,
// policyTargetsNCMove, globalTargetsNC, valueTargetsNCHW, each an .npy v1.0 image
// with a 256-byte header.  Members are stored (zip method 0); numpy's loader and
// the python trainer read stored and deflated members alike.  The file is written
// to "<path>.tmp" and renamed into place, as the reference's writer does.
#include "npzwrite.h"

#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace kc {

struct Crc32Table {
  uint32_t t[256];
  Crc32Table() {
    for(uint32_t i = 0; i < 256; i++) {
      uint32_t c = i;
      for(int k = 0; k < 8; k++)
        c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      t[i] = c;
    }
  }
};

static uint32_t crc32Update(uint32_t crc, const uint8_t* p, size_t n) {
  // a function-local static is initialised once, thread-safely: engine threads of the
  // CLI write files concurrently (the lazily filled table this replaces was a data race,
  // found by tests/test_sanitizers.py::test_cli_sigterm_under_tsan)
  static const Crc32Table tab;
  const uint32_t* table = tab.t;
  crc = ~crc;
  for(size_t i = 0; i < n; i++)
    crc = table[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
  return ~crc;
}

// 256-byte .npy v1.0 header: magic, version, header length 246, dict, space padding, '\n'.
static std::vector<uint8_t> npyHeader(const char* descr, const std::vector<int64_t>& shape) {
  std::vector<uint8_t> h(256, ' ');
  const uint8_t magic[8] = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0};
  memcpy(h.data(), magic, 8);
  h[8] = (uint8_t)((256 - 10) & 0xff);
  h[9] = (uint8_t)((256 - 10) >> 8);
  std::string d = std::string("{'descr':'") + descr + "','fortran_order':False,'shape':(";
  for(size_t i = 0; i < shape.size(); i++) {
    if(i)
      d += ",";
    d += std::to_string(shape[i]);
  }
  if(shape.size() == 1)
    d += ",";
  d += "),}";
  if(d.size() > 256 - 11)
    throw std::invalid_argument("npy header too long");
  memcpy(h.data() + 10, d.data(), d.size());
  h[255] = '\n';
  return h;
}

namespace {
struct Member {
  std::string name;
  std::vector<uint8_t> header;
  const uint8_t* data;
  size_t bytes;
  uint32_t crc;
  uint32_t offset;
};

void put16(std::vector<uint8_t>& b, uint32_t v) {
  b.push_back((uint8_t)v);
  b.push_back((uint8_t)(v >> 8));
}
void put32(std::vector<uint8_t>& b, uint32_t v) {
  for(int i = 0; i < 4; i++)
    b.push_back((uint8_t)(v >> (8 * i)));
}
}  // namespace

void writeNpz(const std::string& path, int n, int X, int Y, const uint8_t* bin, const float* glob,
              const int16_t* pol, const float* gt, const int8_t* val) {
  if(n < 0 || X < 2 || Y < 2)
    throw std::invalid_argument("writeNpz: bad shape");
  const int64_t A = (int64_t)X * Y, pb = (A + 7) / 8, P = 4 * A;
  std::vector<Member> ms = {
    {"binaryInputNCHWPacked", npyHeader("|u1", {n, 15, pb}), bin, (size_t)(n * 15 * pb), 0, 0},
    {"globalInputNC", npyHeader("<f4", {n, 1}), (const uint8_t*)glob, (size_t)n * 4, 0, 0},
    {"policyTargetsNCMove", npyHeader("<i2", {n, 2, P}), (const uint8_t*)pol, (size_t)(n * 2 * P * 2), 0, 0},
    {"globalTargetsNC", npyHeader("<f4", {n, 64}), (const uint8_t*)gt, (size_t)n * 64 * 4, 0, 0},
    {"valueTargetsNCHW", npyHeader("|i1", {n, 5, Y, X}), (const uint8_t*)val, (size_t)(n * 5 * A), 0, 0},
  };
  const std::string tmp = path + ".tmp";
  FILE* f = fopen(tmp.c_str(), "wb");
  if(!f)
    throw std::runtime_error("cannot write " + tmp);
  uint32_t off = 0;
  auto write = [&](const void* p, size_t len) {
    if(len && fwrite(p, 1, len, f) != len) {
      fclose(f);
      throw std::runtime_error("short write to " + tmp);
    }
    off += (uint32_t)len;
  };
  for(Member& m : ms) {
    if(n > 0 && !m.data) {
      fclose(f);
      throw std::invalid_argument("writeNpz: NULL array " + m.name);
    }
    uint32_t crc = crc32Update(0, m.header.data(), m.header.size());
    crc = crc32Update(crc, m.data, m.bytes);
    m.crc = crc;
    m.offset = off;
    const uint32_t size = (uint32_t)(m.header.size() + m.bytes);
    std::vector<uint8_t> lh;
    put32(lh, 0x04034b50u);
    put16(lh, 20);                // version needed
    put16(lh, 0);                 // flags
    put16(lh, 0);                 // method: stored
    put16(lh, 0);                 // mod time
    put16(lh, 0x21);              // mod date (1980-01-01)
    put32(lh, crc);
    put32(lh, size);
    put32(lh, size);
    put16(lh, (uint32_t)m.name.size());
    put16(lh, 0);
    lh.insert(lh.end(), m.name.begin(), m.name.end());
    write(lh.data(), lh.size());
    write(m.header.data(), m.header.size());
    write(m.data, m.bytes);
  }
  const uint32_t cdOff = off;
  std::vector<uint8_t> cd;
  for(const Member& m : ms) {
    const uint32_t size = (uint32_t)(m.header.size() + m.bytes);
    put32(cd, 0x02014b50u);
    put16(cd, 20);
    put16(cd, 20);
    put16(cd, 0);
    put16(cd, 0);
    put16(cd, 0);
    put16(cd, 0x21);
    put32(cd, m.crc);
    put32(cd, size);
    put32(cd, size);
    put16(cd, (uint32_t)m.name.size());
    put16(cd, 0);
    put16(cd, 0);
    put16(cd, 0);
    put16(cd, 0);
    put32(cd, 0);
    put32(cd, m.offset);
    cd.insert(cd.end(), m.name.begin(), m.name.end());
  }
  write(cd.data(), cd.size());
  std::vector<uint8_t> end;
  put32(end, 0x06054b50u);
  put16(end, 0);
  put16(end, 0);
  put16(end, (uint32_t)ms.size());
  put16(end, (uint32_t)ms.size());
  put32(end, (uint32_t)cd.size());
  put32(end, cdOff);
  put16(end, 0);
  write(end.data(), end.size());
  if(fclose(f) != 0)
    throw std::runtime_error("cannot close " + tmp);
  if(rename(tmp.c_str(), path.c_str()) != 0)
    throw std::runtime_error("cannot rename " + tmp + " to " + path);
}

}  // namespace kc
