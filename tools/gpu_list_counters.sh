set -o pipefail
cd /tmp && export TMPDIR=/tmp
mkdir -p $GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 120 rocprofv3 --list-avail > $GRAFT_REPO_ROOT/gpurun_out/avail.txt 2>&1 || true
grep -i "SQ_INSTS\|SQ_INST_\|VALU" $GRAFT_REPO_ROOT/gpurun_out/avail.txt | head -100
