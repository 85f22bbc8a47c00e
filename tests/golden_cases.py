"""Golden-image cases: key -> (scene, width, height, maxBounceCount, samples, frames accumulated in order).
The images in tests/golden/images.npz are CPU-oracle renders (RGB float32), made by tests/golden/make_golden.py."""
CASES = {
    "default_64": ("default", 64, 64, 3, 1, (0,)),
    "default_dielectric_64_f017": ("default_dielectric", 64, 64, 3, 1, (0, 1, 7)),
    "default_emissive_64_2spp": ("default_emissive", 64, 64, 3, 2, (0,)),
    "cornell_c1_256": ("cornell", 256, 256, 1, 1, (0,)),      # BASELINE config 1
    "cornell_64_b4": ("cornell", 64, 64, 4, 1, (0, 1)),
    "atrium_64x36_b4": ("atrium", 64, 36, 4, 1, (0,)),
}
