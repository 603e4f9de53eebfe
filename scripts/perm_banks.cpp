// Host-side LDS bank-conflict model of the permute kernel's tables (development aid).
//   hipcc -std=c++17 -I<csrc> scripts/perm_banks.cpp -L<lib> -ltneqhip -o /tmp/perm_banks
//   /tmp/perm_banks <esz-dtype 0..3> <rank> <seed> [count]
// For random permutations of binary-leg tensors, builds the plan and counts the extra LDS cycles
// of the load-phase ds_writes (groups of 128/esz lanes, bank (a/4) mod 32) and of the
// destination-order reads, per tile, for the vector and the scalar configurations.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <set>
#include <vector>
#include "tq_common.h"
#include "tq_permute.h"

using namespace tq;

static int slot_of(const PermSwz& z, int p) {
  if (z.mode == 0) return p + (p >> 5);
  if (z.mode == 2) return p;
  int x = p;
  for (int q = 0; q < 16; ++q) if ((p >> q) & 1) x ^= z.vsw[q];
  return x;
}

// extra cycles of one group of lanes hitting banks (byte addresses)
static int extra(const std::vector<long>& addrs, int nbanks) {
  std::vector<std::set<long>> per(nbanks);
  for (long a : addrs) per[(a / 4) % nbanks].insert(a / 4);
  size_t mx = 0;
  for (auto& s : per) mx = std::max(mx, s.size());
  return (int)mx - 1;
}

int main(int argc, char** argv) {
  const int dt = atoi(argv[1]), rank = atoi(argv[2]), seed = atoi(argv[3]);
  const int count = argc > 4 ? atoi(argv[4]) : 4;
  const int esz = (int)dtype_size(dt);
  std::mt19937 rng(seed);
  for (int it = 0; it < count; ++it) {
    std::vector<int> perm(rank);
    for (int i = 0; i < rank; ++i) perm[i] = i;
    std::shuffle(perm.begin(), perm.end(), rng);
    std::vector<int64_t> shape(rank, 2), sst(rank);
    for (int i = 0; i < rank; ++i) sst[i] = int64_t(1) << (rank - 1 - perm[i]);
    PermPlan P;
    if (build_perm_plan(dt, rank, shape.data(), sst.data(), &P) != 0) { printf("build failed\n"); return 1; }
    printf("perm %d: kind=%s T=%d vec=%d", it, perm_plan_kind(P), P.tile_elems, P.vec);
    if (P.use_generic) { printf("\n"); continue; }
    const int T = P.tile_elems;
    for (int cfg = 0; cfg < (P.vec > 1 ? 2 : 1); ++cfg) {
      const int vec = cfg ? P.vec : 1;
      const PermSwz& z = cfg ? P.swzv : P.swz1;
      const int64_t* tb = P.tab.data() + (cfg ? 3 * (size_t)T : 0);
      const int G = T / vec;
      const int wgrp = 128 / esz;  // ds_write lanes per banking group
      long wx = 0, wcyc = 0, rx = 0, rcyc = 0;
      for (int b = 0; b < vec; ++b)
        for (int g0 = 0; g0 < G; g0 += wgrp) {
          std::vector<long> a;
          for (int g = g0; g < std::min(G, g0 + wgrp); ++g) {
            const int s = z.mode == 1 ? ((int)tb[G + g] ^ z.vdelta[b]) : ((int)tb[G + g] + z.vdelta[b]);
            a.push_back((long)s * esz);
          }
          wx += extra(a, 32);
          wcyc++;
        }
      const int rb = vec * esz;  // read bytes per lane
      const int rgrp = rb <= 8 ? 32 : 16;
      for (int g0 = 0; g0 < G; g0 += rgrp) {
        std::vector<long> a;
        for (int g = g0; g < std::min(G, g0 + rgrp); ++g) {
          const long base = (long)slot_of(z, vec * g) * esz;
          for (int w = 0; w < rb; w += 4) a.push_back(base + w);
        }
        // each lane's dwords are distinct banks by construction; count max distinct dwords/bank
        rx += extra(a, 64) - (rb > 4 ? 0 : 0);
        rcyc++;
      }
      printf(" | cfg vec%d mode%d: write extra %.2f/grp, read extra %.2f/grp", vec, z.mode,
             (double)wx / wcyc, (double)rx / rcyc);
    }
    printf("\n");
  }
  return 0;
}
