// In-process A/B switches of kernel variants (NOT environment knobs): tools/tower_ab.py flips them
// through the lumen.set_tuning op between interleaved rounds of one process, so a variant is measured
// against its alternative on the same box and warm state.  Production code never changes them.
#pragma once

namespace lumen {

// (r6: the ViT attention split-tail variant lost its A/B -- 6,316 vs 6,339 img/s, 0.301 vs 0.299 ms per
// b512 layer, profiles/r6_tower_ab_tuning_v1.txt, r6_attn_bench_v1.txt -- and was deleted)
enum TuningFlag : int {
  TUNE_LN_MULTI_ROW = 0,      // ln_row_stats: 4 rows per wave for large row counts (1; +0.3 %, same A/B file)
  TUNE_ATTN_CLEAN_CHUNKS = 1, // attn_res_kernel: chunks needing no key mask run the mask-free form (1)
  TUNE_COUNT = 2,
};

int tuning(int flag);
void set_tuning(int flag, int value);

}  // namespace lumen
