// Bounds-checking debug allocator (UNET_GUARD=1): a torch pluggable allocator that surrounds every
// device allocation with 4 KiB guard bands filled with a known byte, plus a check that compares the
// bands of every live allocation after each HIP-library call (unet/_hip/lib.py wraps the calls).
// A kernel that writes past either end of any tensor — ours or torch's — is named at the launch
// that did it, instead of corrupting whichever tensor the caching allocator placed next to it.
// Host code only; debug builds / tests, never the product path.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

namespace {

constexpr size_t kGuard = 4096;
constexpr unsigned char kByte = 0xA7;

struct Block {
  char* base;       // hipMalloc result
  size_t size;      // requested bytes
  size_t total;     // guard + padded size + guard
  int device;
};

std::mutex mu;
std::map<char*, Block> live;   // user pointer -> block
size_t n_alloc = 0, n_bad = 0;
char first_bad[512] = {0};

size_t padded(size_t n) { return (n + kGuard - 1) / kGuard * kGuard; }

// 0 if both bands are intact; otherwise describes the first corrupted byte into msg
int check_block(char* user, const Block& b, char* msg, size_t msglen) {
  static thread_local std::vector<unsigned char> host;
  size_t tail = b.total - kGuard - b.size;
  host.resize(kGuard + tail);
  if (hipMemcpy(host.data(), b.base, kGuard, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  if (hipMemcpy(host.data() + kGuard, user + b.size, tail, hipMemcpyDeviceToHost) != hipSuccess) return 0;
  for (size_t i = 0; i < kGuard; ++i)
    if (host[i] != kByte) {
      snprintf(msg, msglen, "write %zu bytes BEFORE a %zu-byte allocation at %p (byte 0x%02x)", kGuard - i, b.size,
               (void*)user, host[i]);
      return 1;
    }
  for (size_t i = 0; i < tail; ++i)
    if (host[kGuard + i] != kByte) {
      snprintf(msg, msglen, "write at byte %zu PAST the end of a %zu-byte allocation at %p (byte 0x%02x)", i,
               b.size, (void*)user, host[kGuard + i]);
      return 1;
    }
  return 0;
}

}  // namespace

extern "C" {

void* unet_guard_malloc(ssize_t size, int device, hipStream_t stream) {
  (void)stream;
  size_t n = size > 0 ? (size_t)size : 0;
  size_t total = kGuard + padded(n ? n : 1) + kGuard;
  char* base = nullptr;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(device);
  if (hipMalloc(&base, total) != hipSuccess) {
    (void)hipSetDevice(prev);
    return nullptr;
  }
  (void)hipMemset(base, kByte, total);
  (void)hipDeviceSynchronize();
  (void)hipSetDevice(prev);
  std::lock_guard<std::mutex> g(mu);
  live[base + kGuard] = Block{base, n, total, device};
  ++n_alloc;
  return base + kGuard;
}

void unet_guard_free(void* ptr, ssize_t size, int device, hipStream_t stream) {
  (void)size;
  (void)stream;
  (void)device;
  std::lock_guard<std::mutex> g(mu);
  auto it = live.find((char*)ptr);
  if (it == live.end()) return;
  (void)hipDeviceSynchronize();
  char msg[400];
  if (check_block(it->first, it->second, msg, sizeof msg) && n_bad++ == 0)
    snprintf(first_bad, sizeof first_bad, "(found at free) %s", msg);
  (void)hipFree(it->second.base);
  live.erase(it);
}

// Synchronises the device and checks the guard bands of every live allocation.  Returns the number of
// corrupted allocations found since the last call (0 = clean) and describes the first one in msg.
int unet_guard_check(char* msg, int msglen) {
  std::lock_guard<std::mutex> g(mu);
  (void)hipDeviceSynchronize();
  int bad = 0;
  char tmp[400];
  for (auto& kv : live) {
    if (check_block(kv.first, kv.second, tmp, sizeof tmp)) {
      if (bad == 0 && msg && msglen > 0) snprintf(msg, (size_t)msglen, "%s", tmp);
      ++bad;
      (void)hipMemset(kv.second.base, kByte, kGuard);   // re-arm so the next check reports new writes only
      (void)hipMemset(kv.first + kv.second.size, kByte, kv.second.total - kGuard - kv.second.size);
    }
  }
  if (n_bad && bad == 0 && msg && msglen > 0) snprintf(msg, (size_t)msglen, "%s", first_bad);
  int r = bad + (int)n_bad;
  n_bad = 0;
  (void)hipDeviceSynchronize();
  return r;
}

long unet_guard_allocations(void) {
  std::lock_guard<std::mutex> g(mu);
  return (long)n_alloc;
}

}  // extern "C"
