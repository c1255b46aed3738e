set -o pipefail
cd $GRAFT_REPO_ROOT
# r04m: the Schur columns and Gauss-Jordan updates as v_fmac_f64_dpp -- GPU suite,
# factorisation cycles (ftnew = previous commit, ftnew2 = this), bench A/B (new / new2)
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r04m_pytest_gpu.log 2>&1 &&
for v in ftnew ftnew2 ftnew3; do
  for n in 16 32; do
    MPCQ_LIB_VARIANT=exp:$v timeout -k 10 120 python -u tools/factime.py $n > gpurun_out/r04m_factime${n}_$v.txt 2>&1 || exit 1
  done
done &&
for v in new new2 new3 new new2 new3; do
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 300 python -u bench.py --config c4 --steps 3 --warmup 1 --companion 0 --cpu-sample 0 --certify 0 --restatement 0 >> gpurun_out/r04m_bench_c4_ab.txt 2>> gpurun_out/r04m_bench_c4_ab.err || exit 1
  MPCQ_LIB_VARIANT=exp:$v timeout -k 10 300 python -u bench.py --companion 0 --cpu-sample 0 --certify 0 --restatement 0 >> gpurun_out/r04m_bench_c2_ab.txt 2>> gpurun_out/r04m_bench_c2_ab.err || exit 1
done
