bash tools/gpu_session.sh r02s36
