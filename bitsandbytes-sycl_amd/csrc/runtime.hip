// Runtime plumbing behind the C-ABI: the launch stream, the error latch and the
// context/handle entry points the reference's loader probes at import time.
//
//   get_context / get_cusparse     ref:sycl/pythonInterface.cpp:295-296 (cextension.py:82-84, 103)
//   cget_managed_ptr / cprefetch   ref:sycl/pythonInterface.cpp:380-398
//
// The reference has no stream argument (it submits to the device's in-order queue,
// op_quant.cpp:433-434).  Here every launch goes to a per-thread stream that defaults to
// the null stream (PyTorch-ROCm's default stream); `cset_stream` (not in the reference
// ABI, additive) lets the Python layer pass torch.cuda.current_stream().
#include "common.hpp"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include <dlfcn.h>

namespace bnb {

static thread_local hipStream_t g_stream = nullptr;
static std::atomic<int> g_last_error{0};
static std::mutex g_err_mu;
static char g_err_msg[256] = {0};

hipStream_t current_stream() { return g_stream; }

void set_error(int code, const char* what) {
  g_last_error.store(code);
  std::lock_guard<std::mutex> lk(g_err_mu);
  std::snprintf(g_err_msg, sizeof(g_err_msg), "%s (code %d)", what, code);
  if (std::getenv("BNB_HIP_VERBOSE")) std::fprintf(stderr, "[bnb-hip] %s\n", g_err_msg);
}

typedef int (*roctx_push_fn)(const char*);
typedef int (*roctx_pop_fn)();
struct RoctxApi {
  roctx_push_fn push = nullptr;
  roctx_pop_fn pop = nullptr;
  RoctxApi() {
    const char* e = std::getenv("BNB_ROCTX");
    if (!e || std::strcmp(e, "1") != 0) return;
    void* h = dlopen("libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/libroctx64.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return;
    push = reinterpret_cast<roctx_push_fn>(dlsym(h, "roctxRangePushA"));
    pop = reinterpret_cast<roctx_pop_fn>(dlsym(h, "roctxRangePop"));
    if (!push || !pop) push = nullptr, pop = nullptr;
  }
};
static const RoctxApi& roctx_api() {
  static const RoctxApi api;   // thread-safe one-time init
  return api;
}
BnbRange::BnbRange(const char* name) : on(roctx_api().push != nullptr) {
  if (on) roctx_api().push(name);
}
BnbRange::~BnbRange() {
  if (on) roctx_api().pop();
}

}  // namespace bnb

extern "C" {

struct BnbContext {
  int device;
};

void* get_context() {
  auto* c = new BnbContext();
  hipGetDevice(&c->device);
  return c;
}

void* get_cusparse() { return new BnbContext(); }

void* cget_managed_ptr(size_t bytes) {
  void* p = nullptr;
  if (hipMallocManaged(&p, bytes, hipMemAttachHost) != hipSuccess) {
    bnb::set_error(2, "cget_managed_ptr: hipMallocManaged failed");
    return nullptr;
  }
  return p;
}

void cprefetch(void* ptr, size_t bytes, int device) {
  int concurrent = 0;
  hipDeviceGetAttribute(&concurrent, hipDeviceAttributeConcurrentManagedAccess, device);
  if (!concurrent) return;
  hipMemPrefetchAsync(ptr, bytes, device, bnb::current_stream());
}

// --- additive entry points (not in the reference ABI) ---------------------------------
void cset_stream(void* stream) { bnb::g_stream = (hipStream_t)stream; }
void* cget_stream() { return (void*)bnb::g_stream; }

int cget_last_error() { return bnb::g_last_error.exchange(0); }

const char* cget_last_error_message() { return bnb::g_err_msg; }

int cget_abi_version() { return 1; }

// [additive] 1 when roctx ranges are on (BNB_ROCTX=1 and libroctx64 found), else 0
int croctx_enabled() { return bnb::roctx_api().push != nullptr ? 1 : 0; }

}  // extern "C"
