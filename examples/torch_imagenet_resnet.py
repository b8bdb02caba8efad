"""ImageNet ResNet-{50,101,152} + K-FAC (reference: examples/torch_imagenet_resnet.py).

No ImageNet on the target machine: the loader serves synthetic 3x224x224
images with random labels (examples/cnn_utils/datasets.py); the headline
throughput benchmark is bench.py.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from examples import cnn_train  # noqa: E402
from examples.cnn_utils.cli import base_parser, finalize  # noqa: E402

DEFAULTS = dict(model='resnet50', batch_size=32, epochs=55, base_lr=0.0125,
                lr_decay=[25, 35, 40, 45, 50], weight_decay=5e-5, checkpoint_freq=5,
                kfac_update_freq=100, kfac_cov_update_freq=10, damping=0.001,
                label_smoothing=0.1, synthetic_size=1281167, image_size=224)


def main(argv=None):
    args = finalize(base_parser('ImageNet ResNet + K-FAC', DEFAULTS).parse_args(argv))
    return cnn_train.run(args, 'imagenet')


if __name__ == '__main__':
    main()
