"""nvlevelz_amd -- MI355X-native CRC32C block-checksum engine.

Drop-in for the sagitrs/nvlevelz (LevelDB fork) checksum path:
util/crc32c.{h,cc} + port/port_posix_sse.cc, called from
table/table_builder.cc, table/format.cc, db/log_writer.cc and
db/log_reader.cc.  The hot path is hand-written HIP for gfx950 behind the C
ABI in include/nvl_crc32c.h (libnvl_crc32c.so, built in-tree).

Submodules load libnvl_crc32c.so on first use (``nvlevelz_amd.crc32c``
raises if it is missing); ``nvlevelz_amd.launch`` and ``nvlevelz_amd.shard``'s
partition helpers load nothing, so a launcher process can import them
without touching HIP.
"""
import importlib

__all__ = ["crc32c", "framing", "shard", "launch"]


def __getattr__(name):  # PEP 562: `nvlevelz_amd.crc32c` imports on first access
    if name in __all__:
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
