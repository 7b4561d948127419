// drn_host.cc — native host-side helpers (no GPU): CRC32C for TensorBundle checkpoints,
// TFRecord framing (ImageNet shards, tfevents files) and a CIFAR record gatherer.
//
// The reference relied on TF's C++ runtime for these (TensorBundle writer, record readers,
// FixedLengthRecordDataset: SURVEY §2.5 N6/N9/N10); here they are a small C ABI library
// loaded with ctypes. CRC32C uses the SSE4.2 crc32 instruction (8 bytes/instruction) with a
// table-driven fallback.
#include <cstddef>
#include <cstdint>
#include <cstring>
#if defined(__x86_64__)
#include <nmmintrin.h>
#endif

#define DRN_HOST_API extern "C" __attribute__((visibility("default")))

namespace {
struct CrcTable {
  uint32_t t[256];
  CrcTable() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
      t[i] = c;
    }
  }
};

uint32_t crc_sw(const uint8_t* p, size_t n, uint32_t crc) {
  static const CrcTable table;  // thread-safe one-time initialisation (reader threads call this)
  crc = ~crc;
  for (size_t i = 0; i < n; ++i) crc = table.t[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
  return ~crc;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t crc_hw(const uint8_t* p, size_t n, uint32_t crc) {
  uint64_t c = ~crc;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = _mm_crc32_u64(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return ~c32;
}
#endif
}  // namespace

// crc32c(data) continuing from `init` (0 for a fresh value).
DRN_HOST_API uint32_t drn_crc32c(const uint8_t* data, size_t n, uint32_t init) {
#if defined(__x86_64__)
  if (__builtin_cpu_supports("sse4.2")) return crc_hw(data, n, init);
#endif
  return crc_sw(data, n, init);
}

// Table-driven path regardless of the CPU (tests compare it against the SSE4.2 path).
DRN_HOST_API uint32_t drn_crc32c_sw(const uint8_t* data, size_t n, uint32_t init) { return crc_sw(data, n, init); }

DRN_HOST_API uint32_t drn_crc32c_masked(const uint8_t* data, size_t n) {
  const uint32_t c = drn_crc32c(data, n, 0);
  return ((c >> 15) | (c << 17)) + 0xa282ead8u;
}

// Scan a TFRecord buffer: fills offsets/lengths of up to `cap` records, validating both CRCs
// when `check` is set. Returns the number of records, or -(index+1) of the first corrupt one.
DRN_HOST_API long drn_tfrecord_scan(const uint8_t* buf, size_t n, int64_t* offsets, int64_t* lengths, long cap,
                                    int check) {
  size_t pos = 0;
  long cnt = 0;
  while (pos + 12 <= n && cnt < cap) {
    uint64_t len;
    std::memcpy(&len, buf + pos, 8);
    if (check) {
      uint32_t lcrc;
      std::memcpy(&lcrc, buf + pos + 8, 4);
      if (drn_crc32c_masked(buf + pos, 8) != lcrc) return -(cnt + 1);
    }
    if (len > n - pos - 12 || n - pos - 12 - len < 4) return -(cnt + 1);  // no wrap-around on a corrupt length
    if (check) {
      uint32_t dcrc;
      std::memcpy(&dcrc, buf + pos + 12 + len, 4);
      if (drn_crc32c_masked(buf + pos + 12, len) != dcrc) return -(cnt + 1);
    }
    offsets[cnt] = (int64_t)(pos + 12);
    lengths[cnt] = (int64_t)len;
    ++cnt;
    pos += 12 + len + 4;
  }
  return cnt;
}

// Gather CIFAR fixed-length records: rec = [label_bytes][3072 CHW uint8]; writes HWC uint8
// images and int32 labels for the given record indices (label taken at `label_offset`).
DRN_HOST_API void drn_cifar_gather(const uint8_t* data, const int64_t* idx, long n, int record_bytes,
                                   int label_bytes, int label_offset, uint8_t* images_hwc, int32_t* labels) {
  const int H = 32, W = 32, C = 3;
  for (long i = 0; i < n; ++i) {
    const uint8_t* rec = data + (size_t)idx[i] * record_bytes;
    labels[i] = rec[label_offset];
    const uint8_t* chw = rec + label_bytes;
    uint8_t* out = images_hwc + (size_t)i * H * W * C;
    for (int c = 0; c < C; ++c)
      for (int p = 0; p < H * W; ++p) out[p * C + c] = chw[c * H * W + p];
  }
}
