"""MI355X-native RANSAC-F / PnP hot path of bioengstrom/tsbb15-3d-reconstruction-project.

Drop-in modules mirroring the reference surface:
  tsbb15_amd.lab3    fmatrix_stls, fmatrix_residuals, homog
  tsbb15_amd.fun     getFFromLabCode, ransac_f
  tsbb15_amd.ransac  calc_p, calc_r, gen_rnd_indices, norm_p, cart, dpp, dpp_squared,
                     calc_y_prim, ransac_robust
  tsbb15_amd.pnp     p3p, pnp_minimize
  tsbb15_amd.cv      solvePnPRansac, Rodrigues (the tables.py:141-145 call site)
Compute runs in lib/librsamd.so (HIP, gfx950) through ctypes; there is no CPU fallback.
"""
__version__ = "0.1.0"
