"""Build tests/golden/sky_000017_14.npz from the reference's own example
outputs (run in the build container, where /root/reference exists):

  example/000017_14_disp.png  Solver::show_disp's debug view (Solver.cpp:84-93):
                              rows 0..H-1 hold img_l as BGR gray, except row
                              H-1, overwritten by the colormap's first row.
  example/000017_14_sky.png   SkyAreaDetector::detect's output image
                              (imageSkyDetector.cpp:187-191): the detector's
                              input with the sky painted (B,G,R) = (0,0,255).

The detector ran at scale 1 (both images are 1240 wide), so its input is the
debug view's top half with row H-1 taken from the sky image (the sky never
reaches the bottom half of the frame, :326-338), and its mask is the set of
red pixels.  The fixture holds that input and that mask: the reference's own
result for a known input.
"""
import os

import numpy as np
from PIL import Image

REF = "/root/reference/example"
HERE = os.path.dirname(os.path.abspath(__file__))

disp = np.array(Image.open(os.path.join(REF, "000017_14_disp.png")).convert("RGB"))
sky = np.array(Image.open(os.path.join(REF, "000017_14_sky.png")).convert("RGB"))
H = sky.shape[0]
red = (sky[..., 0] == 255) & (sky[..., 1] == 0) & (sky[..., 2] == 0)
img = disp[:H, :, 0].copy()
assert not red[H - 1].any() and (sky[H - 1, :, 0] == sky[H - 1, :, 1]).all()
img[H - 1] = sky[H - 1, :, 0]
# every non-sky pixel of the detector's output image is the input gray
assert (sky[..., 0][~red] == img[~red]).all()
np.savez_compressed(os.path.join(HERE, "sky_000017_14.npz"), image=img,
                    mask=np.where(red, 255, 0).astype(np.uint8))
print("sky pixels", int(red.sum()), "of", red.size)
