#!/bin/bash
# PMC passes for bench.py's roofline (profiles/pmc_summary.json via tools/pmc_summary.py): for each
# per-GPU env count of the strong-scaling curve (65536 / G for G = 1, 2, 4, 8) one rocprofv3 --pmc
# pass per counter group over the 1-GPU bench at that size.  Counter groups stay within one block's
# limits (FETCH_SIZE: 3 TCC, WRITE_SIZE: 2 TCC, so they get separate passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_r02
mkdir -p $OUT
for n in ${SIZES:-65536 32768 16384 8192}; do
  mkdir -p $OUT/n$n
  for part in fetch write issue busy; do
    case $part in
      fetch) grp="FETCH_SIZE" ;;
      write) grp="WRITE_SIZE" ;;
      issue) grp="SQ_WAVES SQ_INSTS_VALU GRBM_GUI_ACTIVE" ;;
      busy)  grp="VALUBusy" ;;
    esac
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/n$n/$part -o p -- \
      python3 bench.py --global-envs $n --steps 10 --warmup 2 --no-cpu-baseline > $OUT/n$n/$part.log 2>&1
    rc=$?
    echo "n=$n $part rc=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
exit 0
