// Host-side IO runtime for mifx: CRC32C (hardware SSE4.2 path + slicing-by-8 fallback) and
// TFRecord framing scan/verify. Reference data path: TFX ExampleGen/Transform gzip TFRecords of
// tf.Example (`airflow-dags/taxi_utils.py:79-83,260-281`).
#include <cstddef>
#include <cstdint>
#include <cstring>

namespace {

uint32_t g_table[8][256];
bool g_init = false;

void init_tables() {
  if (g_init) return;
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : (c >> 1);
    g_table[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; ++i)
    for (int t = 1; t < 8; ++t) g_table[t][i] = (g_table[t - 1][i] >> 8) ^ g_table[0][g_table[t - 1][i] & 0xFF];
  g_init = true;
}

uint32_t crc_sw(const uint8_t* p, size_t n, uint32_t crc) {
  init_tables();
  crc = ~crc;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    v ^= crc;
    crc = g_table[7][v & 0xFF] ^ g_table[6][(v >> 8) & 0xFF] ^ g_table[5][(v >> 16) & 0xFF] ^
          g_table[4][(v >> 24) & 0xFF] ^ g_table[3][(v >> 32) & 0xFF] ^ g_table[2][(v >> 40) & 0xFF] ^
          g_table[1][(v >> 48) & 0xFF] ^ g_table[0][v >> 56];
    p += 8;
    n -= 8;
  }
  while (n--) crc = g_table[0][(crc ^ *p++) & 0xFF] ^ (crc >> 8);
  return ~crc;
}

#if defined(__x86_64__)
__attribute__((target("sse4.2"))) uint32_t crc_hw(const uint8_t* p, size_t n, uint32_t crc) {
  uint64_t c = ~crc;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    c = __builtin_ia32_crc32di(c, v);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = __builtin_ia32_crc32qi(c32, *p++);
  return ~c32;
}
#endif

uint32_t mask(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xA282EAD8u; }

}  // namespace

extern "C" {

uint32_t mifx_crc32c(const char* data, size_t n, uint32_t crc) {
#if defined(__x86_64__)
  static int hw = -1;
  if (hw < 0) hw = __builtin_cpu_supports("sse4.2") ? 1 : 0;
  if (hw) return crc_hw((const uint8_t*)data, n, crc);
#endif
  return crc_sw((const uint8_t*)data, n, crc);
}

// Scan an uncompressed TFRecord buffer. Writes payload offsets/lengths (up to max_records).
// Returns the number of records, or -(1 + index) of the first corrupt record.
long long mifx_tfrecord_scan(const char* buf, size_t len, long long* offsets, long long* lengths,
                             long long max_records, int verify) {
  size_t pos = 0;
  long long n = 0;
  while (pos < len) {
    if (pos + 12 > len) return -(1 + n);
    uint64_t sz;
    std::memcpy(&sz, buf + pos, 8);
    uint32_t hc;
    std::memcpy(&hc, buf + pos + 8, 4);
    if (verify && mask(mifx_crc32c(buf + pos, 8, 0)) != hc) return -(1 + n);
    if (len - pos < 16 || sz > len - pos - 16) return -(1 + n);  // overflow-safe bound (corrupt length)
    if (verify) {
      uint32_t dc;
      std::memcpy(&dc, buf + pos + 12 + sz, 4);
      if (mask(mifx_crc32c(buf + pos + 12, sz, 0)) != dc) return -(1 + n);
    }
    if (n < max_records) {
      offsets[n] = (long long)(pos + 12);
      lengths[n] = (long long)sz;
    }
    ++n;
    pos += 12 + sz + 4;
  }
  return n;
}

}  // extern "C"
