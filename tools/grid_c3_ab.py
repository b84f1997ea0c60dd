#!/usr/bin/env python3
"""Config-3 production-grid parity under precision options of the discriminator (round-4 review item 2).

Each variant runs tests/grid_parity.c3_training_step (the reference's own optimize_parameters at B=16 × 96², nb=23,
bound = 5× the reference's float32 error + 1e-4 floor, unchanged) and prints its worst quantities.
    usage: python tools/grid_c3_ab.py [variant ...]     variants: base gstep_x6 gstep_f32 head_x6 head_f32 bias64
    dgrad_f32 wgrad_f32 trunk_f32 act<A> ...
    (a variant name joins options with '+': e.g. gstep_x6+bias64)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, 'tests'), os.path.join(REPO, 'explorable-super-resolution_old_amd')):
    sys.path.insert(0, p)

import torch  # noqa: E402

OPTS = {'gstep_x6': ('ESR_D_GSTEP_PRECISION', 'x6'), 'gstep_f32': ('ESR_D_GSTEP_PRECISION', 'f32'),
        'head_x6': ('ESR_D_HEAD_PRECISION', 'x6'), 'head_f32': ('ESR_D_HEAD_PRECISION', 'f32')}


def main():
    import grid_parity as GP
    from esr_amd import dconv, engine, train_engine
    dev = torch.device('cuda', 0)
    defaults = (train_engine.DGRAD_X3, train_engine.WGRAD_X3, train_engine.TRUNK_X3, engine.ACT_SCALE)
    for name in sys.argv[1:] or ['base']:
        for k, _ in OPTS.values():
            os.environ.pop(k, None)
        dconv.BIAS_F64 = False
        train_engine.DGRAD_X3, train_engine.WGRAD_X3, train_engine.TRUNK_X3, engine.ACT_SCALE = defaults
        for opt in name.split('+'):
            if opt == 'bias64':
                dconv.BIAS_F64 = True
            elif opt == 'dgrad_f32':  # the generator's residual-block data gradients in exact fp32
                train_engine.DGRAD_X3 = False
            elif opt == 'wgrad_f32':  # its weight gradients on the fp32 kernel
                train_engine.WGRAD_X3 = False
            elif opt == 'trunk_f32':  # its trunk-level (2x / 4x) data gradients in exact fp32
                train_engine.TRUNK_X3 = False
            elif opt.startswith('act'):  # another activation scale of the x3 forward
                engine.ACT_SCALE = float(opt[3:])
            elif opt in OPTS:
                os.environ[OPTS[opt][0]] = OPTS[opt][1]
        r = GP.c3_training_step(dev)
        print('== %s ok %s worst %.4f' % (name, r['ok'], r['worst_frac_of_bound']), flush=True)
        for line in r['lines'][:2]:
            print('   ' + line, flush=True)
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
