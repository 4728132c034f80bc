# Requires R + reticulate + the distributed_amd Python package on the reticulate path.
# The same verbs are covered without R by tests/test_r_package.py (Python mirror).
context("keras verbs")

test_that("the reference model builds, compiles and trains on CPU", {
  skip_if_not(reticulate::py_module_available("distributed_amd"))
  Sys.setenv(DAMD_DEVICE = "cpu")
  mnist <- dataset_mnist()
  x <- array_reshape(mnist$train$x[1:256, , ], c(256, 28, 28, 1)) / 255
  y <- mnist$train$y[1:256]
  model <- keras_model_sequential() %>%
    layer_conv_2d(filters = 32, kernel_size = 3, activation = "relu", input_shape = c(28, 28, 1)) %>%
    layer_max_pooling_2d() %>%
    layer_flatten() %>%
    layer_dense(units = 64, activation = "relu") %>%
    layer_dense(units = 10)
  model %>% compile(loss = tf$keras$losses$SparseCategoricalCrossentropy(from_logits = TRUE),
                    optimizer = tf$keras$optimizers$SGD(learning_rate = 0.001), metrics = "accuracy")
  result <- model %>% fit(x, y, batch_size = 64L, epochs = 3, steps_per_epoch = 2, verbose = 0)
  expect_length(result$metrics$accuracy, 3)
  expect_equal(model$count_params(), 347146)
})

test_that("TF_CONFIG helpers unbox like jsonlite", {
  expect_equal(tf_config("10.0.0.1:8001", 0),
               '{"cluster":{"worker":"10.0.0.1:8001"},"task":{"type":"worker","index":0}}')
  b <- list(address = c("h1:5000", "h2:5000"), partition = 1L)
  expect_match(barrier_tf_config(b), '"worker":\\["h1:8001","h2:8002"\\]')
})
