# Builds libsynctree_hip.so for gfx950 (in-tree, travels to the GPU box) and
# the CPU oracle (test infrastructure).
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC -shared --offload-arch=$(ARCH) -Wall -Wno-unused-result
LIB := riak_ensemble_amd/libsynctree_hip.so
SRC := riak_ensemble_amd/csrc/synctree_hip.hip
DEPS := $(SRC) riak_ensemble_amd/csrc/small_path.h riak_ensemble_amd/csrc/st_kernels.h riak_ensemble_amd/csrc/rehash_win.h riak_ensemble_amd/csrc/md5_dev.h riak_ensemble_amd/csrc/leveldb_fmt.h riak_ensemble_amd/csrc/term_key.h riak_ensemble_amd/csrc/pages.h include/synctree_hip.h

all: $(LIB) oracle

$(LIB): $(DEPS)
	$(HIPCC) $(HIPFLAGS) -o $@ $(SRC)

oracle:
	$(MAKE) -s -C oracle

clean:
	rm -f $(LIB)
	$(MAKE) -s -C oracle clean

.PHONY: all oracle clean
