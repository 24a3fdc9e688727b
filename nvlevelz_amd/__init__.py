"""nvlevelz_amd -- MI355X-native CRC32C block-checksum engine.

Drop-in for the sagitrs/nvlevelz (LevelDB fork) checksum path:
util/crc32c.{h,cc} + port/port_posix_sse.cc, called from
table/table_builder.cc, table/format.cc, db/log_writer.cc and
db/log_reader.cc.  The hot path is hand-written HIP for gfx950 behind the C
ABI in include/nvl_crc32c.h (libnvl_crc32c.so, built in-tree).
"""
from . import crc32c  # noqa: F401  (loads libnvl_crc32c.so; raises if missing)

__all__ = ["crc32c"]
