"""ResNet-18 (BASELINE.json config 4: synthetic 224x224x3) built
with the Keras functional API of this package.

Layout follows the standard ImageNet ResNet-18 (He et al. 2016, "basic" blocks):
Conv 7x7/2 (64) -> BN -> ReLU -> MaxPool 3x3/2 'same' -> 4 stages of 2 BasicBlocks
(64, 128, 256, 512 filters; stride 2 entering stages 2-4, 1x1/2 conv + BN projection
shortcuts) -> GlobalAveragePooling -> Dense(classes) logits.  Convs have no bias
(BN follows), TF 'same' padding, NHWC, Keras default glorot_uniform init.
11,689,512 trainable parameters at 1000 classes (+ 9,600 BN moving statistics).

``widths``/``blocks``/``input_shape`` shrink it for tests; the graph shape stays the same.
"""
from __future__ import annotations


def _basic_block(x, filters, stride, name, layers):
    shortcut = x
    y = layers.Conv2D(filters, 3, strides=stride, padding="same", use_bias=False, name=f"{name}_conv1")(x)
    y = layers.BatchNormalization(epsilon=1.001e-5, name=f"{name}_bn1")(y)
    y = layers.Activation("relu", name=f"{name}_relu1")(y)
    y = layers.Conv2D(filters, 3, padding="same", use_bias=False, name=f"{name}_conv2")(y)
    y = layers.BatchNormalization(epsilon=1.001e-5, name=f"{name}_bn2")(y)
    if stride != 1 or int(x.shape[-1]) != filters:
        shortcut = layers.Conv2D(filters, 1, strides=stride, use_bias=False, name=f"{name}_proj")(x)
        shortcut = layers.BatchNormalization(epsilon=1.001e-5, name=f"{name}_proj_bn")(shortcut)
    y = layers.Add(name=f"{name}_add")([y, shortcut])
    return layers.Activation("relu", name=f"{name}_out")(y)


def resnet18(classes: int = 1000, input_shape=(224, 224, 3), widths=(64, 128, 256, 512), blocks=(2, 2, 2, 2),
             name: str = "resnet18"):
    from ..keras import Model, layers

    inp = layers.Input(shape=input_shape, name="input_1")
    x = layers.Conv2D(widths[0], 7, strides=2, padding="same", use_bias=False, name="conv1_conv")(inp)
    x = layers.BatchNormalization(epsilon=1.001e-5, name="conv1_bn")(x)
    x = layers.Activation("relu", name="conv1_relu")(x)
    x = layers.MaxPooling2D(3, strides=2, padding="same", name="pool1_pool")(x)
    for si, (w, nb) in enumerate(zip(widths, blocks)):
        for bi in range(nb):
            stride = 2 if (si > 0 and bi == 0) else 1
            x = _basic_block(x, w, stride, f"conv{si + 2}_block{bi + 1}", layers)
    x = layers.GlobalAveragePooling2D(name="avg_pool")(x)
    out = layers.Dense(classes, name="predictions")(x)
    return Model(inp, out, name=name)


def compile_resnet(model, learning_rate: float = 0.1, momentum: float = 0.9):
    from .. import keras

    model.compile(loss=keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=keras.optimizers.SGD(learning_rate=learning_rate, momentum=momentum),
                  metrics=["accuracy"])
    return model
