timeout -k 10 300 python scripts/wide_stamps.py 256 && bash scripts/gpu_wide.sh
