// Sanitizer driver for the product's host-core CPU path (csrc/cpu_ops.cpp).  Built by
// tests/test_cpu_sanitizers.py twice -- with -fsanitize=address,undefined and with -fsanitize=thread -- and linked
// against cpu_ops.cpp compiled the same way.  It drives both entry points over ragged, tiny, empty and
// threading-sized inputs at 1 / 3 / 8 / 64 worker threads, from one and from several concurrent host threads, and
// checks every result against a scalar restatement written here (the reference's rule: absmax = fmax over |A|,
// z = A / absmax, left neighbour in the sorted code, one step right iff strictly closer; dequantize code[q] * absmax).
// Exit status 0 and "OK" on success; any mismatch or sanitizer report fails the test.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

extern "C" {
void cquantize_blockwise_cpu_fp32(float* code, float* A, float* absmax, unsigned char* out, long long blocksize,
                                  long long n);
void cdequantize_blockwise_cpu_fp32(float* code, unsigned char* A, float* absmax, float* out, long long blocksize,
                                    long long n);
int cset_cpu_threads(int threads);
}

namespace {

uint32_t lcg(uint32_t& s) {
  s = s * 1664525u + 1013904223u;
  return s;
}

// a sorted signed 256-entry code (the shape of the dynamic map: dense near 0), code[0] = -1
std::vector<float> make_code() {
  std::vector<float> c(256);
  for (int i = 0; i < 256; ++i) {
    const float t = (i - 127.5f) / 127.5f;
    c[i] = t * t * t;
  }
  c[0] = -1.0f;
  c[255] = 1.0f;
  return c;
}

void reference_quantize(const std::vector<float>& code, const std::vector<float>& A, long long bs,
                        std::vector<float>& absmax, std::vector<uint8_t>& q) {
  const long long n = (long long)A.size();
  for (long long s = 0, b = 0; s < n; s += bs, ++b) {
    const long long e = std::min(n, s + bs);
    float m = -FLT_MAX;
    for (long long i = s; i < e; ++i) m = std::fmax(m, std::fabs(A[i]));
    absmax[b] = m;
    for (long long i = s; i < e; ++i) {
      const float z = A[i] / m;
      int idx = 0;
      for (int j = 0; j < 256; ++j)
        if (code[j] <= z) idx = j;
      if (idx < 255 && std::fabs(z - code[idx + 1]) < std::fabs(z - code[idx])) idx += 1;
      q[i] = (uint8_t)idx;
    }
  }
}

struct Case {
  long long n, bs;
  std::vector<float> code, A, am_ref;
  std::vector<uint8_t> q_ref;
  Case(long long n_, long long bs_, uint32_t seed) : n(n_), bs(bs_), code(make_code()), A((size_t)n_) {
    for (auto& v : A) v = ((int32_t)lcg(seed) / 2147483648.0f) * 3.0f;
    if (n > 7) {
      A[3] = 0.0f;
      A[5] = -0.0f;
    }
    const long long nb = n > 0 ? (n + bs - 1) / bs : 0;
    am_ref.assign((size_t)nb + 1, 123.0f);
    q_ref.assign((size_t)n + 1, 0xAB);
    reference_quantize(code, A, bs, am_ref, q_ref);
  }
};

// the product entry points on one case at `threads` workers, checked against the case's reference
int run_case(const Case& c, int threads) {
  const long long n = c.n, bs = c.bs;
  const std::vector<float>& code = c.code;
  const long long nb = n > 0 ? (n + bs - 1) / bs : 0;
  std::vector<float> A = c.A, am((size_t)nb + 1, 123.0f);
  std::vector<uint8_t> q((size_t)n + 1, 0xAB);
  std::vector<float> out((size_t)n + 1, 7.0f);
  const std::vector<float>& am_ref = c.am_ref;
  const std::vector<uint8_t>& q_ref = c.q_ref;
  cset_cpu_threads(threads);
  std::vector<float> code_q = code;
  cquantize_blockwise_cpu_fp32(code_q.data(), A.data(), am.data(), q.data(), bs, n);
  if (n > 0 && code_q[0] != -1.0f) return 1;
  if (std::memcmp(q.data(), q_ref.data(), q.size()) || std::memcmp(am.data(), am_ref.data(), am.size() * 4)) return 2;
  std::vector<float> code_d = code;
  cdequantize_blockwise_cpu_fp32(code_d.data(), q.data(), am.data(), out.data(), bs, n);
  for (long long i = 0; i < n; ++i) {
    const float want = code[q[i]] * am[i / bs];
    if (std::memcmp(&out[i], &want, 4) != 0) return 3;
  }
  if (out[(size_t)n] != 7.0f || q[(size_t)n] != 0xAB || am[(size_t)nb] != 123.0f) return 4;   // nothing past the end
  return 0;
}

}  // namespace

int main() {
  const long long sizes[] = {0, 1, 63, 64, 65, 4097, 1 << 16, (1 << 18) + 37, (1 << 20) + 5};
  const long long blocks[] = {64, 256, 4096};
  const int threads[] = {1, 3, 8, 64};
  int fails = 0, cases = 0;
  for (long long n : sizes)
    for (long long bs : blocks) {
      const Case c(n, bs, (uint32_t)(n * 31 + bs * 7));
      for (int t : threads) {
        const int rc = run_case(c, t);
        ++cases;
        if (rc) {
          std::printf("FAIL n=%lld bs=%lld threads=%d rc=%d\n", n, bs, t, rc);
          ++fails;
        }
      }
    }
  // concurrent callers: four host threads, each with its own buffers, through the shared worker pool setting
  std::vector<Case> cc;
  for (int c = 0; c < 4; ++c) cc.emplace_back((1 << 18) + 11 * c, 64, 1000u + c);
  std::vector<std::thread> callers;
  std::vector<int> rcs(4, -1);
  for (int c = 0; c < 4; ++c)
    callers.emplace_back([c, &rcs, &cc] { rcs[c] = run_case(cc[c], 8); });
  for (auto& th : callers) th.join();
  for (int c = 0; c < 4; ++c) {
    ++cases;
    if (rcs[c]) {
      std::printf("FAIL concurrent caller %d rc=%d\n", c, rcs[c]);
      ++fails;
    }
  }
  cset_cpu_threads(0);
  if (fails) return 1;
  std::printf("OK %d cases\n", cases);
  return 0;
}
