// Permute plan: host-side tile selection + tables, shared by tq_permute and the plan executor.
#pragma once
#include <cstdint>
#include <vector>

#include <hip/hip_runtime.h>

namespace tq {

constexpr int kPermMaxRank = 48;

struct PermOuter {       // iteration over tiles (kernel argument)
  int n;
  int64_t cnt[kPermMaxRank];
  int64_t sstride[kPermMaxRank];
  int64_t dstride[kPermMaxRank];
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
  int tile_elems = 0;
  int64_t n_tiles = 0;
  PermOuter outer{};
  PermGeneric generic{};
  std::vector<int64_t> tab;  // [src offsets | lds slots | dst offsets], each tile_elems long
};

int build_perm_plan(int dtype, int rank, const int64_t* shape, const int64_t* sstrides,
                    PermPlan* plan);
size_t perm_plan_table_bytes(const PermPlan& P);
void perm_plan_pack_table(const PermPlan& P, void* host_buf);
int perm_plan_launch(const PermPlan& P, const void* dtab, const void* src, void* dst, double beta,
                     hipStream_t stream);

}  // namespace tq
