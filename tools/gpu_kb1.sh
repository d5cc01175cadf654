set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out; mkdir -p $O
cd $R
timeout -k 10 200 python -u tools/kbench.py > $O/kb_base.json 2>$O/kb_base.err && cat $O/kb_base.json &&
CODENERF_LIB=$R/code-nerf_amd/libcodenerf_hip_nocomp.so timeout -k 10 200 python -u tools/kbench.py --only dw > $O/kb_nocomp.json 2>>$O/kb_base.err && cat $O/kb_nocomp.json &&
cd /tmp && export TMPDIR=/tmp &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_base -o run -- python3 $R/tools/kbench.py --only dw,copy --reps 3 > $O/pmc_base.log 2>&1 &&
CODENERF_LIB=$R/code-nerf_amd/libcodenerf_hip_nocomp.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_nocomp -o run -- python3 $R/tools/kbench.py --only dw --reps 3 > $O/pmc_nocomp.log 2>&1 && echo done
