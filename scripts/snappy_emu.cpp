// Host emulation of the device snappy decoder (pebble_amd/csrc/snappy_dec.hip.h):
// 64 std::threads run the wave's code in lockstep at every wave primitive.
// Debugging tool only (not part of the product or the tests' checker).
//   /opt/rocm/lib/llvm/bin/clang++ -O1 -std=c++20 -pthread scripts/snappy_emu.cpp -o /tmp/snappy_emu
//   /tmp/snappy_emu in.bin out.bin   (in: a snappy block, uvarint length first)
#include <algorithm>
#include <barrier>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define __device__
#define __forceinline__ inline
template <class T> using lptr = T*;
template <class T> using gptr = T*;
template <class T> T* to_lds_ptr(T* p) { return p; }
template <class T> T* to_glb(T* p) { return p; }
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
struct uint4 { uint32_t x, y, z, w; };
static uint4 make_uint4(uint32_t a, uint32_t b, uint32_t c, uint32_t d) { return uint4{a, b, c, d}; }
constexpr int kWave = 64;
static thread_local int g_lane;
static std::barrier<>* g_bar;
static uint64_t g_slot[64];
static int lane_id() { return g_lane; }
static void wave_sync() { g_bar->arrive_and_wait(); }
template <class T> static T exch(T v, int src) {
  g_bar->arrive_and_wait();
  uint64_t x = 0;
  std::memcpy(&x, &v, sizeof(T));
  g_slot[g_lane] = x;
  g_bar->arrive_and_wait();
  T r;
  uint64_t y = g_slot[src];
  std::memcpy(&r, &y, sizeof(T));
  g_bar->arrive_and_wait();
  return r;
}
template <class T> static T __shfl(T v, int src, int) { return exch(v, src); }
static uint64_t __ballot(int p) {
  g_bar->arrive_and_wait();
  g_slot[g_lane] = p != 0;
  g_bar->arrive_and_wait();
  uint64_t m = 0;
  for (int i = 0; i < 64; i++) m |= g_slot[i] << i;
  g_bar->arrive_and_wait();
  return m;
}
static int emu_readfirstlane(int v) { return exch(v, 0); }  // (int, as the builtin)
static uint32_t emu_alignbyte(uint32_t hi, uint32_t lo, uint32_t r) {
  return uint32_t(((uint64_t(hi) << 32) | lo) >> (8 * (r & 3)));
}
#define __builtin_amdgcn_readfirstlane(x) emu_readfirstlane(x)
#define __builtin_amdgcn_readlane(x, l) exch((x), (l))
#define SN_EMU_SCAN 1
#define __builtin_amdgcn_alignbyte(a, b, c) emu_alignbyte(a, b, c)
#define __builtin_amdgcn_fence(a, b) ((void)0)
#define __builtin_amdgcn_wave_barrier() g_bar->arrive_and_wait()
#define SN_LDS_OR(p, v) __atomic_fetch_or((p), (v), __ATOMIC_RELAXED)
#define SN_T(v)
#define SN_ACC(i, v)
using std::min;
namespace pbl {
namespace phys {
constexpr uint32_t kSnIn = 32768;
constexpr uint32_t kSnQ = 592;
#include "../pebble_amd/csrc/snappy_dec.hip.h"
}  // namespace phys
}  // namespace pbl

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = fopen(argv[1], "rb");
  std::vector<uint8_t> in(1 << 20);  // (zero past the block: the indicator byte's place)
  const size_t n = fread(in.data(), 1, in.size(), f);
  fclose(f);
  uint64_t D = 0;
  uint32_t used = 0;
  for (uint32_t i = 0, s = 0; i < 10; i++, s += 7) {
    D |= uint64_t(in[i] & 0x7f) << s;
    if (in[i] < 0x80) { used = i + 1; break; }
  }
  static pbl::phys::Snap2Lds S;
  // snappy_walk_kernel's lane for this block, then snappy4's decode (or snappy2's)
  const bool walked = pbl::phys::sn4_walkable(uint32_t(n), uint32_t(D)) && !getenv("EMU_NO_WALK");
  if ((!walked && n > pbl::phys::kSnIn) || D > 0xffff) return 3;
  if (!walked) std::memcpy(S.in, in.data(), n);
  std::vector<uint8_t> out(D + 64);
  if (walked) pbl::phys::sn4_walk(in.data(), uint32_t(n), used, uint32_t(D), out.data());
  static pbl::phys::Snap4Lds S4;
  std::barrier<> bar(64);
  g_bar = &bar;
  bool res[64];
  std::vector<std::thread> th;
  for (int l = 0; l < 64; l++)
    th.emplace_back([&, l] {
      g_lane = l;
      res[l] = walked ? pbl::phys::sn4_decode(S4, in.data(), uint32_t(n), uint32_t(D), out.data())
                      : pbl::phys::sn_decode(S, 0, uint32_t(n), used, uint32_t(D), out.data());
    });
  for (auto& t : th) t.join();
  printf("ok %d D %llu\n", int(res[0]), (unsigned long long)D);
  if (argc > 2) {
    FILE* g = fopen(argv[2], "wb");
    fwrite(out.data(), 1, D, g);
    fclose(g);
  }
  return res[0] ? 0 : 1;
}
