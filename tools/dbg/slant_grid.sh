export SGM_HIP_LIB=build/dbg/libsgm_hip.so
echo "grid 256"; timeout -k 10 60 python -u tools/dbg/slant_case.py 51x80_D32 4 | tail -4
echo "grid 256 ldspad 90"; SGM_SLANT_LDSPAD=90 timeout -k 10 60 python -u tools/dbg/slant_case.py 51x80_D32 4 | tail -4
SGM_HIP_LIB=build/slantst/libsgm_hip.so timeout -k 10 100 python tools/slant_stamps.py 2160 3840 256 2
