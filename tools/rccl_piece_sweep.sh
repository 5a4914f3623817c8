for m in ${SIZES:-1073742080 1074790400 1207959552}; do
  r=$(GSORT_FORCE_DIST=1 GSORT_RCCL_MAX_MSG=$m timeout -k 10 120 python3 tests/test_gpu_rccl.py --child-big 2>/dev/null | grep RCCL_BIG)
  echo "$m $r" >> gpurun_out/rccl_sweep.txt
done
