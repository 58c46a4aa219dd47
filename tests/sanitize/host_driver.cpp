// Sanitizer driver (test infrastructure): the library's host-only code -- the matcher and
// SuperPoint weight packers, and every workspace / cache size query over a sweep of shapes
// (ragged, tiny, batched, sharded) -- in a host-only -fsanitize=address,undefined build of
// onepose_amd/csrc (no GPU call is made).  Built and run by tests/test_sanitize.py.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "onepose_hip.h"

namespace {
unsigned s = 2024u;
float frand() {
  s = s * 1664525u + 1013904223u;
  return (float)((s >> 8) / 16777216.0 - 0.5);
}
}  // namespace

int main() {
  if (onepose_abi_version() != 6) return 1;
  // matcher packer
  {
    const int n = onepose_matcher_num_tensors();
    std::vector<std::vector<float>> t(n);
    std::vector<const float*> p(n);
    for (int i = 0; i < n; ++i) {
      if (!onepose_matcher_tensor_name(i)) return 2;
      t[i].resize((size_t)onepose_matcher_tensor_numel(i));
      for (float& x : t[i]) x = frand();
      p[i] = t[i].data();
    }
    std::vector<unsigned char> packed(onepose_matcher_packed_bytes());
    if (onepose_matcher_pack(p.data(), n, packed.data()) != ONEPOSE_OK) return 3;
    // wrong tensor count: must fail cleanly
    if (onepose_matcher_pack(p.data(), n - 1, packed.data()) == ONEPOSE_OK) return 4;
    std::printf("matcher pack: %d tensors, %zu bytes\n", n, packed.size());
  }
  // SuperPoint packer
  {
    // (cin, cout, k) of conv1a .. convDb, the reference's SuperPoint (superpoint.py:147-162)
    const int layers[12][3] = {{1, 64, 3},    {64, 64, 3},   {64, 64, 3},    {64, 64, 3},
                               {64, 128, 3},  {128, 128, 3}, {128, 128, 3},  {128, 128, 3},
                               {128, 256, 3}, {256, 65, 1},  {128, 256, 3},  {256, 256, 1}};
    const int n = onepose_superpoint_num_tensors();
    if (n != 24) return 6;
    std::vector<std::vector<float>> t(n);
    std::vector<const float*> p(n);
    for (int i = 0; i < n; ++i) {
      const int* L = layers[i / 2];
      t[i].resize(i % 2 ? (size_t)L[1] : (size_t)L[1] * L[0] * L[2] * L[2]);
      for (float& x : t[i]) x = frand();
      p[i] = t[i].data();
    }
    std::vector<unsigned char> packed(onepose_superpoint_packed_bytes());
    if (onepose_superpoint_pack(p.data(), n, packed.data()) != ONEPOSE_OK) return 5;
    std::printf("superpoint pack: %d tensors, %zu bytes\n", n, packed.size());
  }
  // size queries
  const int shapes[][4] = {{1, 1, 1, 1},     {1, 256, 512, 8},  {2, 1024, 4096, 8},
                           {1, 1024, 2500, 8}, {32, 1024, 16384, 8}, {1, 2048, 8192, 12},
                           {3, 37, 101, 3}};
  size_t acc = 0;
  for (const auto& sh : shapes) {
    const int B = sh[0], n1 = sh[1], n3 = sh[2], L = sh[3];
    acc += onepose_match_workspace_bytes(B, n1, n3, L, 0) + onepose_match_workspace_bytes(B, n1, n3, L, 1);
    acc += onepose_leaves_prepared_bytes(B, n3, L);
    acc += onepose_object_cache_bytes(n3, L, 0) + onepose_object_cache_bytes(n3, L, ONEPOSE_OBJ_GAT_TABLES);
    acc += onepose_object_prepare_workspace_bytes(n3, L);
    for (int prec = 0; prec <= 3; ++prec) {   // (3: refused, 0 bytes)
      acc += onepose_match_workspace_bytes_ex(B, n1, n3, L, 1, prec);
      acc += onepose_object_cache_bytes_ex(n3, L, ONEPOSE_OBJ_GAT_TABLES, prec);
    }
    for (int world = 1; world <= 3; ++world) {
      acc += onepose_match_sharded_xchg_bytes(B, n1, n3, world);
      for (int r = 0; r < world; ++r) acc += onepose_match_sharded_workspace_bytes(B, n1, n3, world, r, L, 1);
    }
    acc += onepose_pnp_workspace_bytes(B, n1, 10000);
  }
  acc += onepose_superpoint_workspace_bytes(1, 512, 512) + onepose_superpoint_detect_workspace_bytes(2, 480, 640);
  std::printf("size queries ok (%zu)\n", acc);
  return 0;
}
