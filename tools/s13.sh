set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/s13; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; echo "gpu rc=$?"
timeout -k 10 120 ./raytracing_rb_amd/rtx s $O/c2.png scenes/c2_world.yml scenes/c2_camera.yml > $O/cli_c2.log 2>&1; echo "cli rc=$?"
echo rc=$?
