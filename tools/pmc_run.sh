#!/bin/bash
# rocprofv3 PMC passes for one bench config (each counter group in its own pass, no
# tracing domains alongside --pmc). Usage: tools/pmc_run.sh CONFIG OUTDIR [extra bench args]
set -e
cfg=$1; out=$2; shift 2
export TMPDIR=/tmp
mkdir -p "$out"
pass() {
  name=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$out/$name" -o run \
      --pmc "$@" -- python3 bench.py --config "$cfg" --no-cpu-baseline --no-parity \
      --steps 5 --warmup 2 > "$out/$name.log" 2>&1
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE GRBM_GUI_ACTIVE
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM
