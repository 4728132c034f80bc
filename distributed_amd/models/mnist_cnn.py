"""The reference model, exactly as in README.md:58-73 (R) / 292-302 (Python)."""
from __future__ import annotations


def mnist_cnn(filters: int = 32, hidden: int = 64, classes: int = 10, two_conv: bool = False):
    """Conv2D(32,3,relu) -> MaxPool -> Flatten -> Dense(64,relu) -> Dense(10) (347,146 params).

    ``two_conv=True`` builds the "2-conv" variant named by BASELINE.json:7 (an extra
    Conv2D(64,3,relu) after the pool); the reference itself has exactly one conv
    (SURVEY.md §0 discrepancy note)."""
    from ..keras import Sequential, layers

    ls = [layers.Conv2D(filters, 3, activation="relu", input_shape=(28, 28, 1)), layers.MaxPooling2D()]
    if two_conv:
        ls.append(layers.Conv2D(2 * filters, 3, activation="relu"))
    ls += [layers.Flatten(), layers.Dense(hidden, activation="relu"), layers.Dense(classes)]
    return Sequential(ls)


def compile_reference(model, learning_rate: float = 0.001):
    from .. import keras

    model.compile(loss=keras.losses.SparseCategoricalCrossentropy(from_logits=True),
                  optimizer=keras.optimizers.SGD(learning_rate=learning_rate), metrics=["accuracy"])
    return model
