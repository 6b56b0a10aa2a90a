export SGM_HIP_LIB=build/dbg/libsgm_hip.so
echo "down+up"; timeout -k 10 60 python -u tools/dbg/slant_case.py 51x80_D32 4 | tail -4
echo "sweeps+up"; SGM_SLANT_T56SWEEP=1 timeout -k 10 60 python -u tools/dbg/slant_case.py 51x80_D32 4 | tail -4
echo "down+up grid 8"; SGM_SLANT_GRID=8 timeout -k 10 60 python -u tools/dbg/slant_case.py 51x80_D32 4 | tail -4
