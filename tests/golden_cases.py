"""Golden-image cases: key -> (scene, width, height, maxBounceCount, samples, frames accumulated in order).
The images in tests/golden/images.npz are CPU-oracle renders (RGB float32), made by tests/golden/make_golden.py."""
CASES = {
    "default_64": ("default", 64, 64, 3, 1, (0,)),
    "default_dielectric_64_f017": ("default_dielectric", 64, 64, 3, 1, (0, 1, 7)),
    "default_emissive_64_2spp": ("default_emissive", 64, 64, 3, 2, (0,)),
    "cornell_c1_256": ("cornell", 256, 256, 1, 1, (0,)),      # BASELINE config 1
    "cornell_64_b4": ("cornell", 64, 64, 4, 1, (0, 1)),
    "atrium_64x36_b4": ("atrium", 64, 36, 4, 1, (0,)),
    # the reference's own Init scene (mushroom.obj + 4 spheres, start camera; PathTracingRenderer.jai:219-343) with its
    # default knobs (maxBounceCount 3, samples 1, :119-120) and the editor's still-camera frame sequence 1, 3
    "reference_init_64x36": ("reference_init", 64, 36, 3, 1, (1, 3)),
    "reference_init_glass_64x36_2spp": ("reference_init_glass", 64, 36, 3, 2, (0,)),
}
