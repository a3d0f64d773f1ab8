// jit.h — query-shape description and the hipRTC-compiled specialised scan kernels (jit.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <string>
#include <utility>
#include <vector>

namespace pamd {

constexpr int kPartSub = 4;  // partition count / scatter blocks: 4 x 256 threads (one block per CU)
constexpr int kPartCountRatio = 2;  // count-pass blocks per scatter-pass block (count needs little LDS)

struct JitSlot {
  int enc;       // ENC_* (the same in every segment of the batch)
  int type;      // T_* value type
  int bits = 0;  // FIXED_BIT: bit width when every segment of the batch agrees (<= 15), else 0
};
struct JitLeaf {
  int slot;        // -1: reads no column (docId range / bitset / constant)
  int clause;
  int negate;
  uint32_t kinds;  // bit k set: some segment resolves this predicate to LEAF kind k
};
struct JitAcc {
  int op;    // ACC_*
  int slot;
};
struct JitPlan {
  std::vector<JitSlot> slots;
  std::vector<JitLeaf> leaves;  // in DevSegment::leaves order
  int nclauses = 0;
  std::vector<std::pair<int, int64_t>> group;  // (slot, key stride)
  bool any_remap = false;
  std::vector<JitAcc> accs;  // accumulators 1..n (0 is COUNT), in DevQuery acc order
  int64_t num_keys = 1;
  bool lds = false;
  bool bitset = false;
  bool aggregate = true;
  // partitioned GROUP BY (DevPartition): count / scatter / LDS-aggregate kernels instead of one scan
  bool partitioned = false;
  int key_shift = 0;           // keys per partition = 2^key_shift
  int nparts = 0;
  std::vector<int> val_slots;  // record value columns (slots read by accumulators)
  std::vector<int> val_off;    // byte offset of each value column in a record (key u32 at 0)
  int rec_bytes = 0;           // record size, multiple of 8
  int stage_cap = 0;           // scatter: records staged per partition in LDS (0: direct writes)
};
// record layout of a partitioned plan (fills val_off / rec_bytes from val_slots)
void jit_layout_records(JitPlan* p);
// LDS bytes of the scatter pass for a staging capacity
size_t jit_scatter_lds(const JitPlan& p, int cap);
struct JitKernel {
  std::vector<char> image;
  hipModule_t module = nullptr;
  hipFunction_t fn = nullptr;          // pinot_scan_jit, or the partition count pass
  hipFunction_t fn_scatter = nullptr;  // partitioned: scatter pass
  hipFunction_t fn_agg = nullptr;      // partitioned: LDS aggregation of the partitions
};
// record value column j of a partitioned plan: C type of the stored value
const char* jit_val_ctype(const JitSlot& s);
int jit_val_size(const JitSlot& s);

std::string jit_shape_key(const JitPlan& p);
std::string jit_generate(const JitPlan& p);
std::string jit_full_source(const JitPlan& p);
// compiled, loaded kernel for the plan's shape (cached); nullptr + *err when unavailable
JitKernel* jit_get(const JitPlan& p, std::string* err);

}  // namespace pamd
