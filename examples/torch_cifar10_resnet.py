"""CIFAR-10 ResNet-{20,32,44,56,110} + K-FAC (reference: examples/torch_cifar10_resnet.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from examples import cnn_train  # noqa: E402
from examples.cnn_utils.cli import base_parser, finalize  # noqa: E402

DEFAULTS = dict(model='resnet32', batch_size=128, epochs=100, base_lr=0.1, lr_decay=[35, 75, 90],
                weight_decay=5e-4, checkpoint_freq=10, kfac_update_freq=10,
                kfac_cov_update_freq=1, damping=0.003, synthetic_size=50000, image_size=32)


def main(argv=None):
    args = finalize(base_parser('CIFAR-10 ResNet + K-FAC', DEFAULTS).parse_args(argv))
    return cnn_train.run(args, 'cifar')


if __name__ == '__main__':
    main()
