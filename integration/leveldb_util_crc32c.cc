// integration/leveldb_util_crc32c.cc -- drop-in replacement for the
// reference's util/crc32c.cc.
//
// A LevelDB tree compiles this file instead of util/crc32c.cc and stops
// linking port/port_posix_sse.cc (the SSE4.2 accelerator that crc32c.cc calls,
// util/crc32c.cc:299-347, port/port_posix_sse.cc:69-126); every caller of
// util/crc32c.h -- Value, Mask, Unmask are inline there (util/crc32c.h:20-40)
// and reach Extend -- then runs on the engine's C ABI.  The declaration it
// satisfies is the reference's own `extern` one (util/crc32c.h:17), so the
// symbol the rest of the tree links against is unchanged.
//
// oracle/reftests.mk builds the reference's util/crc32c_test.cc and
// db/log_test.cc with this file and libnvl_crc32c.so
// (tests/test_reference_suites.py).
#include "util/crc32c.h"

#include "nvl_crc32c.h"

namespace leveldb {
namespace crc32c {

uint32_t Extend(uint32_t init_crc, const char* data, size_t n) { return nvl_crc32c_extend(init_crc, data, n); }

}  // namespace crc32c
}  // namespace leveldb
