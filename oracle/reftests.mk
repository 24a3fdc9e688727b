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

.PHONY: all
all: $(OUT)/crc32c_test $(OUT)/log_test

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
