// Stub RCCL for the csrc/rccl_direct.cpp sanitizer harness (tools/sanitize/rccl_direct_fuzz.cpp): records the
// arguments of the last ncclAllReduce; count 0xBAD returns an error whose string is longer than the caller's buffer.
// Built with -DNO_ALLREDUCE it exports only ncclGetErrorString (the "symbol missing" path).
#include <cstddef>
#include <cstdint>
#include <string>

static int64_t g_last[7];

extern "C" {
#ifndef NO_ALLREDUCE
int ncclAllReduce(const void* send, void* recv, size_t count, int dtype, int op, void* comm, void* stream) {
  g_last[0] = (int64_t)(intptr_t)send;
  g_last[1] = (int64_t)(intptr_t)recv;
  g_last[2] = (int64_t)count;
  g_last[3] = dtype;
  g_last[4] = op;
  g_last[5] = (int64_t)(intptr_t)comm;
  g_last[6] = (int64_t)(intptr_t)stream;
  return count == 0xBAD ? 3 : 0;
}
const int64_t* stub_last_call() { return g_last; }
#endif
const char* ncclGetErrorString(int) {
  static const std::string s = "stub failure " + std::string(400, 'e');
  return s.c_str();
}
}
