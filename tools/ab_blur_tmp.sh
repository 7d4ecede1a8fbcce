set -e
cd "${GRAFT_REPO_ROOT}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_stereo.py -m gpu -x -q --timeout 120 --timeout-method thread 2>&1 | tail -1
for r in 1 2; do
timeout -k 10 120 python tools/microbench.py --pairs 256 4:0 2>&1 | grep -v amdgpu | tail -1 | sed "s/^/tree(u2): /"
ORBFE_LIB=pyorbslam_amd/_lib/variants/HEAD/liborbfe.so timeout -k 10 120 python tools/microbench.py --pairs 256 4:0 2>&1 | grep -v amdgpu | tail -1 | sed "s/^/HEAD: /"
ORBFE_LIB=pyorbslam_amd/_lib/variants/st4/liborbfe.so timeout -k 10 120 python tools/microbench.py --pairs 256 4:0 2>&1 | grep -v amdgpu | tail -1 | sed "s/^/u4: /"
done
