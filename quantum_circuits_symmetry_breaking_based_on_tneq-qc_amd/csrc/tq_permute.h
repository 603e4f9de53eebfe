// Permute plan: host-side tile selection + tables, shared by tq_permute and the plan executor.
#pragma once
#include <cstdint>
#include <vector>

#include <hip/hip_runtime.h>

namespace tq {

constexpr int kPermMaxRank = 48;

struct PermOuter {       // iteration over tiles (kernel argument)
  int n;
  int all_pow2;          // every cnt is a power of two: decode by shifts (lg) instead of div/mod
  int lg[kPermMaxRank];
  int64_t cnt[kPermMaxRank];
  int64_t sstride[kPermMaxRank];
  int64_t dstride[kPermMaxRank];
};

// LDS image addressing of one kernel configuration (the tile is held in destination order).
//   mode 0 (pad):  slot(p) = p + p / 32                      — scalar kernel, non-power-of-two tiles
//   mode 1 (xor):  slot(p) = p ^ XOR_{bit q of p set} vsw[q]  — power-of-two tiles
//   mode 2 (id):   slot(p) = p                                — vector kernel, non-power-of-two tiles
// vsw[q] only has bits below q (and none below log2(vec)), so the map is a bijection of every
// aligned block onto itself: the destination-order reads stay conflict-free and vectors stay
// contiguous; the vectors are chosen on the host so that the lanes of one ds_write group (the
// load phase, source order) land on distinct banks.
// Element b of a load vector (source-adjacent elements) has slot  slot0 ^ vdelta[b]  (xor) or
// slot0 + vdelta[b]  (pad / id).
struct PermSwz {
  int mode;
  int vsw[16];
  int vdelta[4];
};

struct PermGeneric {     // fallback: one element per thread
  int rank;
  int64_t ext[kPermMaxRank];
  int64_t sstride[kPermMaxRank];
};

struct PermPlan {
  int dtype = 0;
  int64_t numel = 0;
  bool use_generic = true;
  bool idx64 = false;
  int vec = 1;             // elements per lane access of the vector configuration (1, 2 or 4)
  int tile_elems = 0;
  int64_t n_tiles = 0;
  int64_t tile_mul = 1;     // odd: tiles visited in the order t * tile_mul mod n_tiles (n_tiles = 2^k)
  PermOuter outer{};
  PermSwz swz1{};          // scalar configuration
  PermSwz swzv{};          // vector configuration (vec > 1)
  PermGeneric generic{};
  // scalar tables [src offset | lds slot of element 0 | dst offset], tile_elems each (load order
  // for the first two, destination order for the third); with vec > 1 followed by the vector
  // tables of the same layout, tile_elems / vec each.
  std::vector<int64_t> tab;
};

int build_perm_plan(int dtype, int rank, const int64_t* shape, const int64_t* sstrides,
                    PermPlan* plan);
size_t perm_plan_table_bytes(const PermPlan& P);
void perm_plan_pack_table(const PermPlan& P, void* host_buf);
int perm_plan_launch(const PermPlan& P, const void* dtab, const void* src, void* dst, double beta,
                     hipStream_t stream);
// Which kernel a plan launches for 2*sizeof-aligned pointers: "generic", "tiled" or "vecN"
const char* perm_plan_kind(const PermPlan& P);

}  // namespace tq
