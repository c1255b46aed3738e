set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
# r03u: the GPU suite on a build of the final source without the prompt's LDS zeroing
# (-DMPCQ_NO_LDS_ZERO, copied in as libmpcq.so for this run only)
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $O/r03u_pytest_gpu_nozero.log 2>&1
