// jit.h — query-shape description and the hipRTC-compiled specialised scan kernels (jit.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <string>
#include <utility>
#include <vector>

namespace pamd {

struct JitSlot {
  int enc;   // ENC_* (the same in every segment of the batch)
  int type;  // T_* value type
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
};
struct JitKernel {
  std::vector<char> image;
  hipModule_t module = nullptr;
  hipFunction_t fn = nullptr;
};

std::string jit_shape_key(const JitPlan& p);
std::string jit_generate(const JitPlan& p);
std::string jit_full_source(const JitPlan& p);
// compiled, loaded kernel for the plan's shape (cached); nullptr + *err when unavailable
JitKernel* jit_get(const JitPlan& p, std::string* err);

}  // namespace pamd
