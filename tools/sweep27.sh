set -o pipefail
mkdir -p gpurun_out
GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=2 timeout -k 10 120 python -u tools/fill_stamps.py 1000000 125000 > gpurun_out/s27_d2.json || exit 1
GA_FILL_MODE=diag GA_DIAG_COLS_PER_LANE=2 GA_FILL_NWC=8 timeout -k 10 120 python -u tools/fill_stamps.py 1000000 125000 > gpurun_out/s27_d2w8.json || exit 1
rocm-smi --showhw > gpurun_out/s27_hw.txt 2>&1 || true
python -c "import torch; p=torch.cuda.get_device_properties(0); print(p.multi_processor_count)" > gpurun_out/s27_cus.txt 2>&1 || true
