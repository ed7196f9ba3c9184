// Host sanitizer harness for csrc/rccl_direct.cpp (AddressSanitizer + UBSan) against a STUB RCCL library
// (tools/sanitize/rccl_stub.cpp, built as a shared object next to the harness): no GPU, no real RCCL.
// Covers every argument-validation path: collectives before a load, a dlopen failure with a path longer than the
// error buffer (truncated message, no overflow), a library without ncclAllReduce, null communicator / buffer, the
// success path (arguments forwarded: in-place, dtype mapping fp32 -> 7, bf16 -> 9, op sum), and an error return
// whose string is copied into the bounded error buffer.
//   g++ -shared -fPIC tools/sanitize/rccl_stub.cpp -o /tmp/librccl_stub.so
//   g++ -O1 -g -fsanitize=address,undefined tools/sanitize/rccl_direct_fuzz.cpp csrc/rccl_direct.cpp -ldl -o t
//   ./t /tmp/librccl_stub.so /tmp/librccl_nosym.so
#include <dlfcn.h>

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>

extern "C" {
int mifx_rccl_load(const char* path);
const char* mifx_rccl_last_error(void);
int mifx_rccl_allreduce_sum(void* comm, void* buf, size_t n, int dtype, void* stream);
}

static int failures = 0;
#define CHECK(c)                                          \
  do {                                                    \
    if (!(c)) {                                           \
      std::printf("FAILED line %d: %s\n", __LINE__, #c); \
      ++failures;                                         \
    }                                                     \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 3) {
    std::printf("usage: %s <stub rccl .so> <stub without ncclAllReduce .so>\n", argv[0]);
    return 2;
  }
  float buf[8] = {0};
  int comm_dummy = 0;
  CHECK(mifx_rccl_allreduce_sum(&comm_dummy, buf, 8, 0, nullptr) == -1);  // nothing loaded
  const std::string long_path = "/nonexistent/" + std::string(600, 'x') + "/librccl.so";
  CHECK(mifx_rccl_load(long_path.c_str()) == -1);
  CHECK(std::strlen(mifx_rccl_last_error()) < 256 && std::strlen(mifx_rccl_last_error()) > 0);
  CHECK(mifx_rccl_load(argv[2]) == -2);  // loads, but has no ncclAllReduce
  CHECK(std::strstr(mifx_rccl_last_error(), "ncclAllReduce not found") != nullptr);
  CHECK(mifx_rccl_load(argv[1]) == 0);
  CHECK(mifx_rccl_load(argv[1]) == 0);  // idempotent
  CHECK(mifx_rccl_allreduce_sum(nullptr, buf, 8, 0, nullptr) == -1);
  CHECK(mifx_rccl_allreduce_sum(&comm_dummy, nullptr, 8, 0, nullptr) == -1);
  // the stub records its arguments
  void* h = dlopen(argv[1], RTLD_NOW | RTLD_NOLOAD);
  CHECK(h != nullptr);
  auto last = (const int64_t* (*)())dlsym(h, "stub_last_call");
  CHECK(last != nullptr);
  int stream_dummy = 0;
  CHECK(mifx_rccl_allreduce_sum(&comm_dummy, buf, 8, 0, &stream_dummy) == 0);
  const int64_t* a = last();
  CHECK(a[0] == (int64_t)(intptr_t)buf && a[1] == (int64_t)(intptr_t)buf);  // in place
  CHECK(a[2] == 8 && a[3] == 7 && a[4] == 0);                               // n, ncclFloat32, ncclSum
  CHECK(a[5] == (int64_t)(intptr_t)&comm_dummy && a[6] == (int64_t)(intptr_t)&stream_dummy);
  CHECK(mifx_rccl_allreduce_sum(&comm_dummy, buf, 4, 1, nullptr) == 0);
  CHECK(last()[3] == 9);  // ncclBfloat16
  // n == 0xBAD makes the stub fail with a long error string: copied bounded
  CHECK(mifx_rccl_allreduce_sum(&comm_dummy, buf, 0xBAD, 0, nullptr) == 3);
  CHECK(std::strncmp(mifx_rccl_last_error(), "ncclAllReduce: stub failure", 27) == 0);
  CHECK(std::strlen(mifx_rccl_last_error()) < 256);
  std::printf("%d failures\n", failures);
  return failures != 0;
}
