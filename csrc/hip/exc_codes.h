// Exception classes of a replay (mirror of fks::ExcCode, csrc/include/fks/types.hpp
// and policy/bytecode.py `Exc`): what the reference's `evaluate_policy_standalone`
// turns into score 0, plus the engine-internal "ask the next engine" codes.
#pragma once

#include "jit_env.h"

namespace fksd {

enum ExcCode : int32_t {
  EXC_NONE = 0, EXC_ZERO_DIVISION = 1, EXC_VALUE = 2, EXC_OVERFLOW = 3, EXC_TYPE = 4,
  EXC_INDEX = 5, EXC_ALLOC = 6, EXC_NAME = 7, EXC_UNSUPPORTED = 100, EXC_BUDGET = 101, EXC_INVARIANT = 102,
  EXC_TIMEOUT = 103,   // two-wave kernel: a wave stopped hearing from its partner (spin cap; timing, not the program)
  EXC_EVENTS = 104,    // the replay passed the caller's event budget (RowNativeArgs::max_events): not scored
};

}  // namespace fksd
