# Launch / data targets (ref Makefile, run_approx_coding.sh, data_prepare.sh) for one MI355X node.
#
# One process per GPU: NGPUS=1 runs main.py directly, NGPUS>1 launches torchrun (RCCL over xGMI).
# N_PROCS keeps the reference meaning: 1 master + N_PROCS-1 logical workers, spread over the GPUs.
# Every run target passes all 13 positional arguments (the reference Makefile passed 10 and
# main.py rejected them).

N_PROCS ?= 9
N_STRAGGLERS ?= 1
N_COLLECT ?= 6
N_PARTITIONS ?= 4
PARTIAL_CODED ?= 0
ADD_DELAY ?= 0
UPDATE_RULE ?= AGD
DATA_FOLDER ?= ./straggdata/
IS_REAL ?= 0
DATASET ?= artificial
N_ROWS ?= 1000000
N_COLS ?= 1000
NGPUS ?= 1
EXTRA ?=
PORT ?= 29500

PY ?= python
ifeq ($(NGPUS),1)
RUN = $(PY) main.py
else
RUN = $(PY) -m torch.distributed.run --nnodes=1 --nproc-per-node $(NGPUS) --master-addr 127.0.0.1 --master-port $(PORT) main.py
endif
ARGS = $(N_PROCS) $(N_ROWS) $(N_COLS) $(DATA_FOLDER) $(IS_REAL) $(DATASET)

.PHONY: build test test-gpu bench generate_random_data arrange_real_data naive cyccoded repcoded approxcoded \
        avoidstragg partialrepcoded partialcyccoded sanitize

build:
	PYTORCH_ROCM_ARCH=gfx950 $(PY) tools/build_ext.py

test:
	$(PY) -m pytest tests -x -q -m "not gpu"

test-gpu:
	$(PY) -m pytest tests -x -q -m gpu

sanitize:
	bash tools/sanitize_host.sh

bench:
ifeq ($(NGPUS),1)
	$(PY) bench.py --gpus 1
else
	$(PY) -m torch.distributed.run --nnodes=1 --nproc-per-node $(NGPUS) --master-addr 127.0.0.1 --master-port $(PORT) bench.py --gpus $(NGPUS)
endif

generate_random_data:
	$(PY) -m erasurehead_amd.data.generate $(N_PROCS) $(N_ROWS) $(N_COLS) $(DATA_FOLDER) $(N_STRAGGLERS) $(N_PARTITIONS) $(PARTIAL_CODED)

arrange_real_data:
	$(PY) -m erasurehead_amd.data.prepare $(N_PROCS) $(DATA_FOLDER) $(DATASET) $(N_STRAGGLERS) $(N_PARTITIONS) $(PARTIAL_CODED)

naive:
	$(RUN) $(ARGS) 0 $(N_STRAGGLERS) 0 0 $(N_COLLECT) $(ADD_DELAY) $(UPDATE_RULE) $(EXTRA)

cyccoded:
	$(RUN) $(ARGS) 1 $(N_STRAGGLERS) 0 0 $(N_COLLECT) $(ADD_DELAY) $(UPDATE_RULE) $(EXTRA)

repcoded:
	$(RUN) $(ARGS) 1 $(N_STRAGGLERS) 0 1 $(N_COLLECT) $(ADD_DELAY) $(UPDATE_RULE) $(EXTRA)

avoidstragg:
	$(RUN) $(ARGS) 1 $(N_STRAGGLERS) 0 2 $(N_COLLECT) $(ADD_DELAY) $(UPDATE_RULE) $(EXTRA)

approxcoded:
	$(RUN) $(ARGS) 1 $(N_STRAGGLERS) 0 3 $(N_COLLECT) $(ADD_DELAY) $(UPDATE_RULE) $(EXTRA)

partialrepcoded:
	$(RUN) $(ARGS) 1 $(N_STRAGGLERS) $(N_PARTITIONS) 1 $(N_COLLECT) $(ADD_DELAY) $(UPDATE_RULE) $(EXTRA)

partialcyccoded:
	$(RUN) $(ARGS) 1 $(N_STRAGGLERS) $(N_PARTITIONS) 0 $(N_COLLECT) $(ADD_DELAY) $(UPDATE_RULE) $(EXTRA)
