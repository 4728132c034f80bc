# Python side: the distributed_amd package (reticulate, delay-loaded so library() is cheap).
# The reference drives TensorFlow through the R 'tensorflow'/'keras' packages and
# reticulate (reference README.md:28-40, 46-75); here the same verbs drive distributed_amd.

.damd <- new.env(parent = emptyenv())

.py <- function() {
  if (is.null(.damd$mod)) {
    .damd$mod <- reticulate::import("distributed_amd", delay_load = FALSE)
    .damd$r <- reticulate::import("distributed_amd.r_api", delay_load = FALSE)
  }
  .damd$mod
}

.r <- function() {
  .py()
  .damd$r
}

#' The `tf` namespace object: tf$keras$..., tf$distribute$experimental$MultiWorkerMirroredStrategy()
#' @export
tf <- NULL

#' The Keras namespace (tf$keras)
#' @export
keras <- NULL

.onLoad <- function(libname, pkgname) {
  tf <<- reticulate::import("distributed_amd", delay_load = TRUE)
  keras <<- reticulate::import("distributed_amd.keras", delay_load = TRUE)
}

#' @export
tf_version <- function() .r()$tf_version()

#' Nothing to install: the framework ships its own native runtime (kept for script parity).
#' @export
install_tensorflow <- function(...) invisible(.r()$install_tensorflow())
