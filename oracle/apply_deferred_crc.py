"""TEST INFRASTRUCTURE (oracle/Makefile): apply INTEGRATION.md §5's edit to
the reference's table/table_builder.cc at build time, writing the result to
oracle/_ref/ (git-ignored build output, like the objects compiled from
/root/reference; nothing is committed).  The edit: TableBuilder::WriteRawBlock
(table_builder.cc:175-193) leaves a block's trailer CRC at zero when its file
seals trailers itself (nvl::shims::DefersBlockCrc, include/nvl_leveldb_shims.h),
instead of computing crc32c::Value/Extend/Mask per block.

    python3 apply_deferred_crc.py SRC DST
"""
import re
import sys

src, dst = sys.argv[1], sys.argv[2]
text = open(src).read()
# the three statements computing and encoding the trailer CRC
pat = re.compile(r"(?P<ind>[ \t]*)uint32_t crc = crc32c::Value\(block_contents\.data\(\), block_contents\.size\(\)\);\n"
                 r"[ \t]*crc = crc32c::Extend\(crc, trailer, 1\);[^\n]*\n"
                 r"[ \t]*EncodeFixed32\(trailer\+1, crc32c::Mask\(crc\)\);\n")
m = list(pat.finditer(text))
assert len(m) == 1, f"expected the WriteRawBlock CRC statements once, found {len(m)}"
ind = m[0].group("ind")
new = (f"{ind}uint32_t crc = 0;  // the file seals the trailers in one batch (nvl_leveldb_shims.h)\n"
       f"{ind}if (!nvl::shims::DefersBlockCrc(r->file)) {{\n"
       f"{ind}  crc = crc32c::Mask(crc32c::Extend(crc32c::Value(block_contents.data(), block_contents.size()),\n"
       f"{ind}                                   trailer, 1));\n"
       f"{ind}}}\n"
       f"{ind}EncodeFixed32(trailer+1, crc);\n")
text = text[:m[0].start()] + new + text[m[0].end():]
inc = '#include "table/format.h"\n'
assert inc in text
text = text.replace(inc, inc + '#include "nvl_leveldb_shims.h"\n', 1)
open(dst, "w").write(text)
