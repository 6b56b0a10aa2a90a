# per-pass slant stamps: real, no courier, no courier + hot memory
for v in slantst pnocst phot; do
  echo "== $v"
  SGM_HIP_LIB=build/$v/libsgm_hip.so timeout -k 10 100 python tools/slant_stamps.py 2160 3840 256 2 || exit 1
done
