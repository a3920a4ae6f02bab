for b in 0 256 32 16 48; do
  if [ $b = 0 ]; then echo "r0: $(timeout -k 10 120 python -u tools/ring_ab.py 3 2>&1 | grep -v amdgpu | head -1)" || exit 1
  else echo "r$b: $(SG2HIP_LIB=tools/diag_libs/libsg2hip_r$b.so timeout -k 10 120 python -u tools/ring_ab.py 3 2>&1 | grep -v amdgpu | head -1)" || exit 1; fi
done
