# probe: H pair on a second stream beside the top-down slanted pass
for c in hd256 4k256; do
  bash tools/ab.sh $c 1 stereo_matching_amd/libsgm_hip.so build/ovl/libsgm_hip.so || exit 1
  for f in 0.5 0.625 0.75; do
    echo "SGM_DOWN_FRAC=$f"; SGM_DOWN_FRAC=$f bash tools/ab.sh $c 1 build/ovl/libsgm_hip.so || exit 1
  done
  echo "H first, 0.5"; SGM_H_FIRST=1 SGM_DOWN_FRAC=0.5 bash tools/ab.sh $c 1 build/ovl/libsgm_hip.so || exit 1
done
