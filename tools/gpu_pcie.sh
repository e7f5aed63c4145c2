set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 120 python tools/pcie_probe.py > gpurun_out/pcie.json 2>gpurun_out/pcie.err; echo sdma rc=$?; cat gpurun_out/pcie.json
HSA_ENABLE_SDMA=0 timeout -k 10 120 python tools/pcie_probe.py > gpurun_out/pcie_blit.json 2>gpurun_out/pcie_blit.err; echo blit rc=$?; cat gpurun_out/pcie_blit.json
