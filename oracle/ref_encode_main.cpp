// ref_encode_main.cpp -- TEST INFRASTRUCTURE ONLY.
//
// A tiny driver (our own code) around the reference's public encoder class,
// Shared/HuffmanEncoder.{hpp,cpp}, which oracle/Makefile compiles unmodified
// from /root/reference into oracle/_ref/ref_encode. It performs the same two
// calls HuffmanUtil::encodeHuffman makes (Shared/HuffmanUtil.cpp:1077-1117):
// HuffmanEncoder::encode, then lookupBufferBitOffsets at every
// stride-th symbol. HuffmanUtil.cpp itself is not built (it needs Apple's
// <simd/simd.h> through AAPLShaderTypes.h; see oracle/README.md).
//
// usage: ref_encode <symbols.bin> <stride> <out_prefix>
//   writes <out_prefix>.canon (256 B), .codes (encoder bytes incl. its 2 zero
//   bytes), .offsets (u32 little-endian, one per stride symbols) and .header
//   (the 8-byte container header encode() emits and the renderer drops).
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "HuffmanEncoder.hpp"

static bool write_file(const std::string &path, const void *data, size_t n) {
  FILE *f = std::fopen(path.c_str(), "wb");
  if (!f) return false;
  bool ok = std::fwrite(data, 1, n, f) == n;
  std::fclose(f);
  return ok;
}

int main(int argc, char **argv) {
  if (argc != 4) {
    std::fprintf(stderr, "usage: %s <symbols.bin> <stride> <out_prefix>\n", argv[0]);
    return 2;
  }
  FILE *f = std::fopen(argv[1], "rb");
  if (!f) return 3;
  std::vector<uint8_t> in;
  uint8_t buf[1 << 16];
  size_t got;
  while ((got = std::fread(buf, 1, sizeof(buf), f)) > 0) in.insert(in.end(), buf, buf + got);
  std::fclose(f);
  const long stride = std::strtol(argv[2], nullptr, 10);
  if (in.empty() || stride <= 0) return 4;

  HuffmanEncoder enc;
  std::vector<uint8_t> header, canon, codes;
  if (!enc.encode(in, header, canon, codes)) return 5;

  std::vector<uint32_t> query;
  for (size_t i = 0; i + (size_t)stride <= in.size(); i += (size_t)stride) query.push_back((uint32_t)i);
  std::vector<uint32_t> offsets = enc.lookupBufferBitOffsets(query);

  const std::string p = argv[3];
  if (!write_file(p + ".canon", canon.data(), canon.size())) return 6;
  if (!write_file(p + ".codes", codes.data(), codes.size())) return 6;
  if (!write_file(p + ".offsets", offsets.data(), offsets.size() * sizeof(uint32_t))) return 6;
  if (!write_file(p + ".header", header.data(), header.size())) return 6;
  return 0;
}
