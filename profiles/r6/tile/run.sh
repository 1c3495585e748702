set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tile
P=cuda-hip-mpi-heat-equation-test_amd/_native/tile_probe
timeout -k 10 120 $P 32768 > gpurun_out/tile/probe_32768.json 2> gpurun_out/tile/probe_32768.err
rc=$?; echo "probe 32768 rc=$rc"; cat gpurun_out/tile/probe_32768.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 $P 16384 > gpurun_out/tile/probe_16384.json 2> gpurun_out/tile/probe_16384.err
rc=$?; echo "probe 16384 rc=$rc"; tail -4 gpurun_out/tile/probe_16384.json
