"""Model zoo: toy linear problem (reference parity), MNIST CNN, ResNet-50, BERT-base."""
from .resnet import resnet50, ResNet, synthetic_batch  # noqa: F401
from .bert import BertConfig, BertForPreTraining  # noqa: F401
from .mnist import MnistCNN, synthetic_mnist  # noqa: F401
