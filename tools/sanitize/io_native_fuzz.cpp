// Host sanitizer harness for csrc/io_native.cpp (AddressSanitizer + UBSan; GPU sanitizers are not
// available on the MI355X pool). Builds valid TFRecord buffers, then scans them intact, truncated at
// every length, and with random header/payload corruption (with and without CRC verification),
// checking that the scanner never reads out of bounds and reports corruption.
//   g++ -O1 -g -fsanitize=address,undefined -fno-omit-frame-pointer -std=c++17 \
//       tools/sanitize/io_native_fuzz.cpp csrc/io_native.cpp -o /tmp/io_fuzz && /tmp/io_fuzz
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

extern "C" {
uint32_t mifx_crc32c(const char* data, size_t n, uint32_t crc);
long long mifx_tfrecord_scan(const char* buf, size_t len, long long* offsets, long long* lengths,
                             long long max_records, int verify);
}

static uint32_t masked(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xA282EAD8u; }

static void append_record(std::vector<char>& out, const std::vector<char>& payload) {
  uint64_t n = payload.size();
  char hdr[8];
  std::memcpy(hdr, &n, 8);
  uint32_t hc = masked(mifx_crc32c(hdr, 8, 0));
  uint32_t dc = masked(mifx_crc32c(payload.data(), payload.size(), 0));
  out.insert(out.end(), hdr, hdr + 8);
  out.insert(out.end(), (char*)&hc, (char*)&hc + 4);
  out.insert(out.end(), payload.begin(), payload.end());
  out.insert(out.end(), (char*)&dc, (char*)&dc + 4);
}

int main() {
  std::mt19937_64 rng(1234);
  // CRC32C known answer: "123456789" -> 0xE3069283
  if (mifx_crc32c("123456789", 9, 0) != 0xE3069283u) {
    std::printf("crc32c KAT failed\n");
    return 1;
  }
  int failures = 0;
  for (int trial = 0; trial < 200; ++trial) {
    std::vector<char> buf;
    const int nrec = 1 + (int)(rng() % 6);
    for (int r = 0; r < nrec; ++r) {
      std::vector<char> p(rng() % 300);
      for (auto& c : p) c = (char)rng();
      append_record(buf, p);
    }
    std::vector<long long> off(16), len(16);
    // exact-size copies so any over-read is caught by ASan
    std::vector<char> exact(buf.begin(), buf.end());
    if (mifx_tfrecord_scan(exact.data(), exact.size(), off.data(), len.data(), 16, 1) != nrec) ++failures;
    for (size_t cut = 0; cut < buf.size(); cut += 1 + rng() % 7) {
      std::vector<char> t(buf.begin(), buf.begin() + cut);
      long long r0 = mifx_tfrecord_scan(t.data(), t.size(), off.data(), len.data(), 16, 0);
      long long r1 = mifx_tfrecord_scan(t.data(), t.size(), off.data(), len.data(), 16, 1);
      (void)r0;
      if (cut > 0 && r1 >= 0 && r1 == nrec) ++failures;  // truncated data cannot scan completely
    }
    for (int k = 0; k < 20; ++k) {
      std::vector<char> t(buf.begin(), buf.end());
      t[rng() % t.size()] ^= (char)(1 + rng() % 255);
      if (k % 4 == 0 && t.size() >= 8) {  // hostile length field
        uint64_t huge = ~0ull - (rng() % 64);
        std::memcpy(t.data(), &huge, 8);
      }
      mifx_tfrecord_scan(t.data(), t.size(), off.data(), len.data(), 16, 0);
      long long rv = mifx_tfrecord_scan(t.data(), t.size(), off.data(), len.data(), 16, 1);
      if (rv == nrec) ++failures;  // a flipped byte must be detected when verifying
    }
  }
  std::printf("io_native fuzz: %d failures\n", failures);
  return failures ? 1 : 0;
}
