// In-process A/B switches of kernel variants (NOT environment knobs): tools/tower_ab.py flips them
// through the lumen.set_tuning op between interleaved rounds of one process, so a variant is measured
// against its alternative on the same box and warm state.  Production code never changes them.
#pragma once

namespace lumen {

enum TuningFlag : int {
  TUNE_ATTN_SPLIT_TAIL = 0,   // attn_res_kernel: split the ragged last query block over the waves (1)
  TUNE_LN_MULTI_ROW = 1,      // ln_row_stats: 4 rows per wave for large row counts (1)
  TUNE_COUNT = 2,
};

int tuning(int flag);
void set_tuning(int flag, int value);

}  // namespace lumen
