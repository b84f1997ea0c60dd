"""Training and Z-optimisation parity at the PRODUCTION grids, so that the shape-dependent launch
choices (x3 weight-gradient split-K, per-RRDB gradient scales, discriminator tile / split-K modes) run exactly as in
bench_train.py / bench_zopt.py.  The checks live in tests/grid_parity.py (bench.py reports the same numbers).

* Config 3: SRRaGANModel.optimize_parameters, B=16 × 96² LR, RRDB-23, latent, CEM train mode (the D sees the
  unpadded HR), WGAN-GP — two micro-steps (a D step, then a D + G step) against the REFERENCE's own
  optimize_parameters run on the same seeded weights and batches in float64 and float32
  (tests/golden/make_golden_train.py c3): every G and D parameter gradient of the second step through K seeded
  random projections (relative L2 distance to the float64 run within 5× the reference's own float32 distance plus a
  floor of 1e-4), the logged D outputs / losses / gradient penalty and the D BatchNorm buffers as in
  test_gpu_train_loop.py.
* Config 5: dL/dZ, dL/dLR and the output of images 0 and 7 of a B=8 × 128² batch through the latent RRDB-23 + CEM
  (eval, pre-pad) against the reference's autograd, with the ×4 kernel of the reference's own KernelGAN
  post-processing (CEM margins 22 / 88, G at 172²: SURVEY §8's reading; make_golden.py c5grid_kgan) and with the
  learned 13×13 kernel of the CEM fixtures (margins 13 / 52; make_golden.py c5grid)."""
import pytest

import grid_parity as GP

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('precision,fold', [('x3', 'product'), ('f32', 'product'), ('f32', 'rowmajor'),
                                            ('f32', 'f64')])
def test_c3_training_step_at_production_grid(gpu_device, precision, fold):
    """x3 and exact fp32; the fp32 step also with the upsampler's folded weights summed in the two other legal orders
    of profiles/r4_c3_fold_order.txt (row-major: 125 % of the single-run bound in round 4), each gated on the
    ensemble bound (grid_parity: the plain and the rounding-perturbed reference float32 runs)."""
    with GP.upsampler_fold(fold):
        r = GP.c3_training_step(gpu_device, precision)
    print('\n'.join(r['lines']))
    print('worst quantity at %.1f %% of its bound (%.1f %% of the single-run bound)' % (
        100 * r['worst_frac_of_bound'], 100 * r.get('worst_frac_of_single_run_bound', float('nan'))))
    assert r['ok'], r['fails']


@pytest.mark.parametrize('kernel', ['kgan', 'learned13'])
@pytest.mark.parametrize('precision', ['x3', 'f32'])
def test_c5_z_gradients_at_production_grid(gpu_device, precision, kernel):
    r = GP.c5_z_gradients(gpu_device, precision, kernel)
    print('\n'.join(r['lines']))
    assert r['ok'], r['fails']
