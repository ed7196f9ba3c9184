// Force-included into every mifx native library by mifx/ops/build.py (-include): the sha256 prefix of the sources
// and flags the library was built from, as a marker string in the binary and through mifx_src_hash(), so the
// loader (mifx/ops/_lib.py) can refuse a library that does not match the sources next to it.
#pragma once
#ifdef MIFX_SRC_HASH_VALUE
extern "C" __attribute__((visibility("default"), used)) const char* mifx_src_hash() {
  static const char marker[] = "MIFX_SRC_HASH=" MIFX_SRC_HASH_VALUE;
  return marker + 14;
}
#endif
