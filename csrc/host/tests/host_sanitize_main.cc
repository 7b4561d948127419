// host_sanitize_main.cc — drives every entry point of drn_host.cc under AddressSanitizer +
// UndefinedBehaviorSanitizer (sanitizers on host code; GPU ASan is not available
// on the MI355X pool). Built and run by tests/test_host_sanitizers.py:
//   g++ -fsanitize=address,undefined -fno-omit-frame-pointer -g drn_host.cc host_sanitize_main.cc
// Exercises exact-size heap buffers, so any out-of-bounds read in the TFRecord scanner or the
// CIFAR gather (e.g. on truncated or corrupt input) aborts the run; the same driver built with
// -fsanitize=thread checks the concurrent first use of the CRC table (the data pipeline's
// reader threads call these functions in parallel).
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

extern "C" {
uint32_t drn_crc32c(const uint8_t* data, size_t n, uint32_t init);
uint32_t drn_crc32c_sw(const uint8_t* data, size_t n, uint32_t init);
uint32_t drn_crc32c_masked(const uint8_t* data, size_t n);
long drn_tfrecord_scan(const uint8_t* buf, size_t n, int64_t* offsets, int64_t* lengths, long cap, int check);
void drn_cifar_gather(const uint8_t* data, const int64_t* idx, long n, int record_bytes, int label_bytes,
                      int label_offset, uint8_t* images_hwc, int32_t* labels);
}

static int g_fail = 0;
#define CHECK(c)                                                     \
  do {                                                               \
    if (!(c)) {                                                      \
      std::fprintf(stderr, "CHECK failed line %d: %s\n", __LINE__, #c); \
      g_fail = 1;                                                    \
    }                                                                \
  } while (0)

static void put_record(std::vector<uint8_t>& out, const std::vector<uint8_t>& payload) {
  uint8_t hdr[12];
  const uint64_t len = payload.size();
  std::memcpy(hdr, &len, 8);
  const uint32_t lcrc = drn_crc32c_masked(hdr, 8);
  std::memcpy(hdr + 8, &lcrc, 4);
  out.insert(out.end(), hdr, hdr + 12);
  out.insert(out.end(), payload.begin(), payload.end());
  const uint32_t dcrc = drn_crc32c_masked(payload.data(), payload.size());
  const uint8_t* d = reinterpret_cast<const uint8_t*>(&dcrc);
  out.insert(out.end(), d, d + 4);
}

// a heap copy of exactly n bytes, so ASan's redzone sits right behind the last byte
static uint8_t* exact(const std::vector<uint8_t>& v, size_t n) {
  uint8_t* p = static_cast<uint8_t*>(std::malloc(n ? n : 1));
  if (n) std::memcpy(p, v.data(), n);
  return p;
}

int main() {
  // CRC32C check value and hardware/software agreement over odd lengths and offsets
  const char* s = "123456789";
  CHECK(drn_crc32c(reinterpret_cast<const uint8_t*>(s), 9, 0) == 0xE3069283u);
  std::vector<uint8_t> rnd(4200);
  uint32_t x = 12345;
  for (auto& b : rnd) b = (uint8_t)((x = x * 1103515245u + 12345u) >> 24);
  for (size_t off : {0, 1, 3, 7}) {
    for (size_t n : {0, 1, 7, 8, 9, 63, 4096}) {
      uint8_t* p = exact(std::vector<uint8_t>(rnd.begin() + off, rnd.begin() + off + n), n);
      CHECK(drn_crc32c(p, n, 0) == drn_crc32c_sw(p, n, 0));
      std::free(p);
    }
  }

  // concurrent first use of the software CRC table from several threads
  {
    std::vector<std::thread> ths;
    std::vector<uint32_t> res(8);
    for (int t = 0; t < 8; ++t)
      ths.emplace_back([&, t]() { res[t] = drn_crc32c_sw(rnd.data() + t, 1000, 0); });
    for (auto& th : ths) th.join();
    for (int t = 0; t < 8; ++t) CHECK(res[t] == drn_crc32c(rnd.data() + t, 1000, 0));
  }

  // TFRecord: three records scanned from an exact-size buffer
  std::vector<uint8_t> buf;
  put_record(buf, std::vector<uint8_t>(5, 1));
  put_record(buf, std::vector<uint8_t>(0, 0));
  put_record(buf, std::vector<uint8_t>(300, 7));
  int64_t offs[8], lens[8];
  uint8_t* b = exact(buf, buf.size());
  CHECK(drn_tfrecord_scan(b, buf.size(), offs, lens, 8, 1) == 3);
  CHECK(lens[0] == 5 && lens[1] == 0 && lens[2] == 300);
  CHECK(drn_tfrecord_scan(b, buf.size(), offs, lens, 2, 1) == 2);  // capacity respected
  std::free(b);
  // every truncation: never reads past the end, reports the first incomplete record
  for (size_t n = 0; n < buf.size(); ++n) {
    uint8_t* t = exact(buf, n);
    const long r = drn_tfrecord_scan(t, n, offs, lens, 8, 1);
    CHECK(r >= -3 && r <= 2);
    std::free(t);
  }
  // corrupt length fields (no CRC check): huge / wrapping lengths must not be followed
  for (uint64_t bad : {uint64_t(1) << 40, ~uint64_t(0), ~uint64_t(0) - 11, uint64_t(buf.size())}) {
    std::vector<uint8_t> c = buf;
    std::memcpy(c.data(), &bad, 8);
    uint8_t* t = exact(c, c.size());
    CHECK(drn_tfrecord_scan(t, c.size(), offs, lens, 8, 0) == -1);
    CHECK(drn_tfrecord_scan(t, c.size(), offs, lens, 8, 1) == -1);
    std::free(t);
  }
  // corrupt payload byte: caught by the data CRC
  {
    std::vector<uint8_t> c = buf;
    c[12 + 2] ^= 0x40;
    uint8_t* t = exact(c, c.size());
    CHECK(drn_tfrecord_scan(t, c.size(), offs, lens, 8, 1) == -1);
    std::free(t);
  }

  // CIFAR gather: CHW -> HWC, last record of an exact-size file
  const int rb = 3073, nrec = 4;
  std::vector<uint8_t> recs((size_t)rb * nrec);
  for (size_t i = 0; i < recs.size(); ++i) recs[i] = (uint8_t)(i * 7);
  uint8_t* data = exact(recs, recs.size());
  const int64_t idx[2] = {3, 0};
  std::vector<uint8_t> img(2 * 32 * 32 * 3);
  int32_t labels[2];
  drn_cifar_gather(data, idx, 2, rb, 1, 0, img.data(), labels);
  CHECK(labels[0] == recs[(size_t)3 * rb] && labels[1] == recs[0]);
  CHECK(img[5 * 3 + 2] == recs[(size_t)3 * rb + 1 + 2 * 1024 + 5]);  // pixel 5, channel 2 of record 3
  std::free(data);

  std::printf(g_fail ? "host sanitizer driver: FAILED\n" : "host sanitizer driver: OK\n");
  return g_fail;
}
