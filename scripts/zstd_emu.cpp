// Host emulation of the device zstd decoder (pebble_amd/csrc/zstd_dec.hip.h):
// 64 std::threads run the wave's code in lockstep at every wave primitive
// (wave_sync, __shfl, __ballot), so decoder bugs can be found on the CPU.
// Debugging tool only (not part of the product or the tests' checker).
//   g++ -O1 -std=c++20 -pthread scripts/zstd_emu.cpp -o /tmp/zstd_emu
//   /tmp/zstd_emu in.bin out.bin   (in: Pebble zstd block = uvarint + frames)
#include <barrier>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>
#include <algorithm>

#define __device__
#define __constant__ static const
#define __forceinline__ inline
template <class T> using lptr = T*;
template <class T> using gptr = T*;
template <class T> T* to_lds_ptr(T* p) { return p; }
template <class T> T* to_glb(T* p) { return p; }
constexpr int kWave = 64;
static thread_local int g_lane;
static std::barrier<>* g_bar;
static uint64_t g_slot[64];
static int lane_id() { return g_lane; }
static void wave_sync() { g_bar->arrive_and_wait(); }
template <class T> static T __shfl(T v, int src, int) {
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
static uint64_t __ballot(int p) {
  g_bar->arrive_and_wait();
  g_slot[g_lane] = p != 0;
  g_bar->arrive_and_wait();
  uint64_t m = 0;
  for (int i = 0; i < 64; i++) m |= g_slot[i] << i;
  g_bar->arrive_and_wait();
  return m;
}
static void __builtin_amdgcn_fence(int, const char*) {}
static void __builtin_amdgcn_wave_barrier() { g_bar->arrive_and_wait(); }
using std::min;
#define PBL_ZSTD_EMU_STEP() g_bar->arrive_and_wait()
#define PBL_ZSTD_EMU_MID() g_bar->arrive_and_wait()

#include "../pebble_amd/csrc/zstd_dec.hip.h"

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = fopen(argv[1], "rb");
  std::vector<uint8_t> in(1 << 22);
  size_t n = fread(in.data(), 1, in.size(), f);
  fclose(f);
  uint64_t D = 0;
  uint32_t used = 0;
  for (uint32_t i = 0, s = 0; i < 10; i++, s += 7) {
    D |= uint64_t(in[i] & 0x7f) << s;
    if (in[i] < 0x80) { used = i + 1; break; }
  }
  static pbl::zstd::Lds L;
  std::vector<uint8_t> out(D + 64);
  const bool lds = n - used <= pbl::zstd::kIn && D <= pbl::zstd::kOut;
  if (lds) std::memcpy(L.in, in.data() + used, n - used);
  std::barrier<> bar(64);
  g_bar = &bar;
  uint32_t res[64];
  std::vector<std::thread> th;
  for (int l = 0; l < 64; l++)
    th.emplace_back([&, l] {
      g_lane = l;
      if (lds)
        res[l] = pbl::zstd::decode_frames(L, pbl::zstd::LIn{L.in}, 0, uint32_t(n - used), pbl::zstd::LOut{L.out},
                                          uint32_t(D));
      else
        res[l] = pbl::zstd::decode_frames(L, pbl::zstd::GIn{in.data() + used}, 0, uint32_t(n - used),
                                          pbl::zstd::GOut{out.data()}, uint32_t(D));
    });
  for (auto& t : th) t.join();
  if (lds) std::memcpy(out.data(), L.out, D);
  printf("status %u (lane 63: %u) D %llu path %s\n", res[0], res[63], (unsigned long long)D, lds ? "lds" : "global");
  if (argc > 2) {
    FILE* g = fopen(argv[2], "wb");
    fwrite(out.data(), 1, D, g);
    fclose(g);
  }
  return res[0];
}
