DETECT_LEAKS=0 bash tools/gpu_asan.sh r02s28
