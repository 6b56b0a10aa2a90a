# top-down pass's share of the CUs (n/8) beside the H pair, per frame size
for L in stereo_matching_amd/libsgm_hip.so build/dg3/libsgm_hip.so build/dg5/libsgm_hip.so build/dg6/libsgm_hip.so; do
  echo "== $L"
  SGM_HIP_LIB=$L timeout -k 10 200 python tools/slant_sizes.py 1080x1920x256x2 2160x3840x256x2 2160x3840x256x1 2160x3840x128x2 || exit 1
done
