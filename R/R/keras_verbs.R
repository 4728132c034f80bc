# Keras verbs with the argument names of the R keras package (reference README.md:46-75).
# Integer-valued doubles (R's default numeric) are passed as Python ints where Keras
# needs ints (filters, units, kernel sizes, batch size, epochs).

.int <- function(x) if (is.null(x)) NULL else as.integer(x)
.ints <- function(x) if (is.null(x)) NULL else reticulate::tuple(as.list(as.integer(x)))

.tag <- function(model) {
  class(model) <- unique(c("distributed_amd_model", class(model)))
  model
}

#' @export
dataset_mnist <- function(path = "mnist.npz") .r()$dataset_mnist(path)

#' Row-major reshape (same semantics as reticulate::array_reshape)
#' @export
array_reshape <- function(x, dim, order = c("C", "F")) reticulate::array_reshape(x, dim, order = match.arg(order))

#' @export
keras_model_sequential <- function(layers = NULL, name = NULL) .tag(.r()$keras_model_sequential(layers, name))

#' @export
layer_conv_2d <- function(object = NULL, filters, kernel_size, strides = c(1L, 1L), padding = "valid",
                          activation = NULL, use_bias = TRUE, input_shape = NULL, name = NULL, ...) {
  .r()$layer_conv_2d(object, filters = .int(filters), kernel_size = .ints(kernel_size), strides = .ints(strides),
                     padding = padding, activation = activation, use_bias = use_bias,
                     input_shape = .ints(input_shape), name = name, ...)
}

#' @export
layer_max_pooling_2d <- function(object = NULL, pool_size = c(2L, 2L), strides = NULL, padding = "valid",
                                 name = NULL) {
  .r()$layer_max_pooling_2d(object, pool_size = .ints(pool_size), strides = .ints(strides), padding = padding,
                            name = name)
}

#' @export
layer_average_pooling_2d <- function(object = NULL, pool_size = c(2L, 2L), strides = NULL, padding = "valid",
                                     name = NULL) {
  .r()$layer_average_pooling_2d(object, pool_size = .ints(pool_size), strides = .ints(strides), padding = padding,
                                name = name)
}

#' @export
layer_flatten <- function(object = NULL, input_shape = NULL, name = NULL) {
  .r()$layer_flatten(object, name = name, input_shape = .ints(input_shape))
}

#' @export
layer_dense <- function(object = NULL, units, activation = NULL, use_bias = TRUE, input_shape = NULL, name = NULL,
                        ...) {
  .r()$layer_dense(object, units = .int(units), activation = activation, use_bias = use_bias,
                   input_shape = .ints(input_shape), name = name, ...)
}

#' @export
layer_dropout <- function(object = NULL, rate, name = NULL) .r()$layer_dropout(object, rate = rate, name = name)

#' @export
layer_batch_normalization <- function(object = NULL, name = NULL, ...) {
  .r()$layer_batch_normalization(object, name = name, ...)
}

#' @export
layer_activation <- function(object = NULL, activation, name = NULL) {
  .r()$layer_activation(object, activation = activation, name = name)
}

#' @export
compile <- function(object, optimizer = NULL, loss = NULL, metrics = NULL, ...) {
  invisible(.tag(.r()$compile(object, optimizer = optimizer, loss = loss, metrics = metrics, ...)))
}

#' fit() returns the History; `result$metrics$accuracy` works as in the R keras package
#' (reference README.md:218-220).
#' @export
fit <- function(object, x = NULL, y = NULL, batch_size = NULL, epochs = 10, verbose = 1, callbacks = NULL,
                steps_per_epoch = NULL, validation_split = 0, validation_data = NULL, shuffle = TRUE,
                initial_epoch = 0, ...) {
  h <- .r()$fit(object, x = x, y = y, batch_size = .int(batch_size), epochs = .int(epochs), verbose = .int(verbose),
                callbacks = callbacks, steps_per_epoch = .int(steps_per_epoch), validation_split = validation_split,
                validation_data = validation_data, shuffle = shuffle, initial_epoch = .int(initial_epoch), ...)
  structure(list(params = reticulate::py_to_r(h$params),
                 metrics = lapply(reticulate::py_to_r(h$history), unlist),
                 py = h), class = "keras_training_history")
}

#' @export
evaluate <- function(object, x, y, batch_size = NULL, verbose = 1) {
  .r()$evaluate(object, x, y, batch_size = .int(batch_size), verbose = .int(verbose))
}

#' @export
predict.distributed_amd_model <- function(object, x, batch_size = NULL, ...) {
  .r()$predict(object, x, batch_size = .int(batch_size))
}

#' @export
save_model_hdf5 <- function(object, filepath, overwrite = TRUE, include_optimizer = TRUE) {
  invisible(.r()$save_model_hdf5(object, filepath, overwrite = overwrite, include_optimizer = include_optimizer))
}

#' @export
load_model_hdf5 <- function(filepath, compile = TRUE) .tag(.r()$load_model_hdf5(filepath, compile = compile))

#' @export
save_model_weights_hdf5 <- function(object, filepath) invisible(.r()$save_model_weights_hdf5(object, filepath))

#' @export
load_model_weights_hdf5 <- function(object, filepath) invisible(.r()$load_model_weights_hdf5(object, filepath))

#' base64enc::base64encode(file) / base64decode(string) equivalents (reference README.md:240-246)
#' @export
base64encode <- function(what) .r()$base64encode(what)

#' @export
base64decode <- function(what) .r()$base64decode(what)
