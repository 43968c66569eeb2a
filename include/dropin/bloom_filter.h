// Drop-in replacement for jackdent/cs265-lsm-tree src/bloom_filter.h: the
// whole file.  src/bloom_filter.cpp is deleted; the filter is bloomhip's.
#include <cstdint>
#include "types.h"
#include <bloomhip_bloom_filter.hpp>
