# The reference's sparklyr barrier example (README.md:171-223) on one MI355X node:
# sdf_len/spark_apply/collect come from distributedamd (no Spark needed), one worker per GPU.
library(distributedamd)

res <- sdf_len(NULL, 8, repartition = 8) %>%
  spark_apply(function(df, barrier) {
    tryCatch({
      library(distributedamd)
      Sys.setenv(TF_CONFIG = barrier_tf_config(barrier))
      strategy <- tf$distribute$experimental$MultiWorkerMirroredStrategy()
      num_workers <- length(barrier$address)
      batch_size <- 64L * num_workers
      mnist <- dataset_mnist()
      x_train <- array_reshape(mnist$train$x, c(nrow(mnist$train$x), 28, 28, 1)) / 255
      y_train <- mnist$train$y
      with(strategy$scope(), {
        model <- keras_model_sequential() %>%
          layer_conv_2d(filters = 32, kernel_size = 3, activation = "relu", input_shape = c(28, 28, 1)) %>%
          layer_max_pooling_2d() %>%
          layer_flatten() %>%
          layer_dense(units = 64, activation = "relu") %>%
          layer_dense(units = 10)
        model %>% compile(loss = tf$keras$losses$SparseCategoricalCrossentropy(from_logits = TRUE),
                          optimizer = tf$keras$optimizers$SGD(learning_rate = 0.001), metrics = "accuracy")
      })
      result <- model %>% fit(x_train, y_train, batch_size = batch_size, epochs = 3, steps_per_epoch = 5)
      as.character(max(result$metrics$accuracy))
    }, error = function(e) e$message)
  }, barrier = TRUE, columns = c(address = "character")) %>%
  collect()
print(res)
