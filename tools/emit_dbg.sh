for d in 0 1 2 4 3 7; do
  BIC_LIB_PATH=binary-image-compression_amd/lib/libbic_stamps.so BIC_EMIT_DBG=$d timeout -k 10 120 python3 bench.py --no-cpu --no-check --separate > gpurun_out/dbg_$d.log 2>&1 || exit 1
done
