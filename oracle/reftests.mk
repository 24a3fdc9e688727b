# oracle/reftests.mk -- the reference's own CRC32C and log test suites linked
# against the engine: util/crc32c_test.cc (4 tests) and db/log_test.cc
# (38 tests) compiled straight from $(REF) (read-only, nothing copied), with
# integration/leveldb_util_crc32c.cc in place of util/crc32c.cc +
# port/port_posix_sse.cc, against nvlevelz_amd/libnvl_crc32c.so.
#
# util/testharness.cc's TmpDir() names Env::Default(), so util/env_posix.cc
# and the NVM library objects it constructs are linked too (neither suite
# calls it: Env::Default() builds a 1500 MB NVM_Library, util/env_posix.cc:895-902,
# which is what segfaults here).
#
#   make -f oracle/reftests.mk        (from the repo root; outputs in oracle/_ref/reftests)
REF  ?= /root/reference
CXX  ?= g++
ROOT := $(abspath $(dir $(lastword $(MAKEFILE_LIST)))/..)
OUT  := $(ROOT)/oracle/_ref/reftests
LIB  := $(ROOT)/nvlevelz_amd/libnvl_crc32c.so
FLAGS := -O1 -w -std=c++11 -I$(REF) -I$(REF)/include -I$(REF)/nvm_library -I$(ROOT)/include \
         -DLEVELDB_PLATFORM_POSIX -DOS_LINUX -DLEVELDB_ATOMIC_PRESENT

COMMON := util/testharness.cc util/env.cc util/env_posix.cc util/status.cc port/port_posix.cc util/logging.cc \
          util/coding.cc nvm_library/global.cc nvm_library/nvm_filesystem.cc nvm_library/nvm_manager.cc \
          nvm_library/nvm_allocator.cc nvm_library/nvm_file.cc nvm_library/nvm_options.cc nvm_library/sysnvm.cc
obj = $(addprefix $(OUT)/,$(subst /,__,$(1:.cc=.o)))

# The SSTable pinning suites: table/table_test.cc (Harness
# block/table/memtable/DB round trips, table_test.cc:648-836) and
# db/corruption_test.cc (corruption_test.cc:236-358: TableFile,
# TableFileIndexData, CompactionInputErrorParanoid, ...) need the whole
# engine -- DB::Open on Env::Default() -- so every library source the
# reference's own build lists (build_detect_platform:171-183: db/ util/ table/
# nvm_library/ minus tests, benches and tools) is compiled here, at -O0: at -O2
# Env::Default() crashes on NVM_Manager::write_zero falling off its end (UB,
# DESIGN.md §9).  util/crc32c.cc and port/port_posix_sse.cc are NOT among
# them: the forwarder replaces both.
ENGINE := $(filter-out %test.cc %_bench.cc db/db_bench.old.cc db/db_bench_original.cc db/leveldbutil.cc \
            util/crc32c.cc,$(patsubst $(REF)/%,%,$(wildcard $(REF)/db/*.cc $(REF)/util/*.cc $(REF)/table/*.cc \
            $(REF)/nvm_library/*.cc))) port/port_posix.cc
ENGINE_TEST := util/testharness.cc util/testutil.cc
EFLAGS := -O0 -g0 -w -std=c++11 -I$(REF) -I$(REF)/include -I$(REF)/nvm_library -I$(ROOT)/include \
          -DLEVELDB_PLATFORM_POSIX -DOS_LINUX -DLEVELDB_ATOMIC_PRESENT -pthread
eobj = $(addprefix $(OUT)/e_,$(subst /,__,$(1:.cc=.o)))

.PHONY: all tables
all: $(OUT)/crc32c_test $(OUT)/log_test
tables: $(OUT)/table_test $(OUT)/corruption_test $(OUT)/table_test.ref $(OUT)/corruption_test.ref

$(OUT)/e_%.o: | $(OUT)
	$(CXX) $(EFLAGS) -c $(REF)/$(subst __,/,$*).cc -o $@

$(OUT)/e_forwarder.o: $(ROOT)/integration/leveldb_util_crc32c.cc | $(OUT)
	$(CXX) $(EFLAGS) -c $< -o $@

$(OUT)/table_test: $(call eobj,table/table_test.cc $(ENGINE) $(ENGINE_TEST)) $(OUT)/e_forwarder.o $(LIB)
	$(CXX) -o $@ $(filter %.o,$^) -L$(dir $(LIB)) -lnvl_crc32c -Wl,-rpath,$(dir $(LIB)) -lpthread

$(OUT)/corruption_test: $(call eobj,db/corruption_test.cc $(ENGINE) $(ENGINE_TEST)) $(OUT)/e_forwarder.o $(LIB)
	$(CXX) -o $@ $(filter %.o,$^) -L$(dir $(LIB)) -lnvl_crc32c -Wl,-rpath,$(dir $(LIB)) -lpthread

$(OUT):
	mkdir -p $@

$(OUT)/%.o: | $(OUT)
	$(CXX) $(FLAGS) -c $(REF)/$(subst __,/,$*).cc -o $@

$(OUT)/forwarder.o: $(ROOT)/integration/leveldb_util_crc32c.cc | $(OUT)
	$(CXX) $(FLAGS) -c $< -o $@


$(OUT)/crc32c_test: $(call obj,util/crc32c_test.cc $(COMMON)) $(OUT)/forwarder.o $(LIB)
	$(CXX) -o $@ $(filter %.o,$^) -L$(dir $(LIB)) -lnvl_crc32c -Wl,-rpath,$(dir $(LIB)) -lpthread

$(OUT)/log_test: $(call obj,db/log_test.cc db/log_reader.cc db/log_writer.cc $(COMMON)) $(OUT)/forwarder.o $(LIB)
	$(CXX) -o $@ $(filter %.o,$^) -L$(dir $(LIB)) -lnvl_crc32c -Wl,-rpath,$(dir $(LIB)) -lpthread

# Control builds: the same suites on the reference's OWN util/crc32c.cc +
# port/port_posix_sse.cc (SSE4.2), to tell a failure of the fork itself from
# one of the drop-in (tests/test_reference_suites.py compares the two).
$(OUT)/e_ref_crc32c.o: $(REF)/util/crc32c.cc | $(OUT)
	$(CXX) $(EFLAGS) -c $< -o $@
$(OUT)/e_ref_port_sse.o: $(REF)/port/port_posix_sse.cc | $(OUT)
	$(CXX) $(EFLAGS) -msse4.2 -DLEVELDB_PLATFORM_POSIX_SSE -c $< -o $@
$(OUT)/table_test.ref: $(call eobj,table/table_test.cc $(ENGINE) $(ENGINE_TEST)) $(OUT)/e_ref_crc32c.o \
                       $(OUT)/e_ref_port_sse.o
	$(CXX) -o $@ $(filter %.o,$^) -lpthread
$(OUT)/corruption_test.ref: $(call eobj,db/corruption_test.cc $(ENGINE) $(ENGINE_TEST)) $(OUT)/e_ref_crc32c.o \
                            $(OUT)/e_ref_port_sse.o
	$(CXX) -o $@ $(filter %.o,$^) -lpthread
