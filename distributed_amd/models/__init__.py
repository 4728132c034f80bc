"""Model zoo: the reference MNIST CNN (README.md:58-68) and ResNet-18 (BASELINE.json:10)."""
from .mnist_cnn import mnist_cnn, compile_reference  # noqa: F401
from .resnet import resnet18, compile_resnet  # noqa: F401
