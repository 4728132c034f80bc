# TF_CONFIG helpers (reference README.md:84-113, 180-183) and a local replacement for
# sparklyr's sdf_len() %>% spark_apply(barrier = TRUE) %>% collect() (README.md:171-223).

#' jsonlite::toJSON(list(cluster = list(worker = workers), task = list(type = 'worker',
#' index = index)), auto_unbox = TRUE)
#' @export
tf_config <- function(workers, index) {
  as.character(jsonlite::toJSON(list(cluster = list(worker = workers),
                                     task = list(type = "worker", index = as.integer(index))),
                                auto_unbox = TRUE))
}

#' The Spark closure's TF_CONFIG: executor hosts, ports base_port + 1..n (README.md:181)
#' @export
barrier_tf_config <- function(barrier, base_port = 8000L) {
  hosts <- gsub(":[0-9]+$", "", barrier$address)
  tf_config(paste(hosts, base_port + seq_along(barrier$address), sep = ":"), barrier$partition)
}

#' A local "Spark DataFrame" of n rows in n partitions (one per worker / GPU).
#' @export
sdf_len <- function(sc = NULL, length, repartition = length) {
  structure(list(n = as.integer(length), partitions = as.integer(repartition)), class = "damd_sdf")
}

#' Gang-scheduled barrier apply: one Rscript worker per partition, all started at once,
#' each with barrier = list(address = c(...), partition = i) and DAMD_LOCAL_RANK = i (its
#' GPU); returns `f(df, barrier)` per partition in partition order.
#'
#' Gang semantics are those of the Python launcher (distributed_amd.launch.launch_command,
#' tested there): the workers' exit statuses are polled, the first failure kills every
#' surviving worker (no orphan keeps a GPU) and the whole gang restarts, up to
#' `max_restarts` times (Spark barrier-stage semantics).  An error raised by `f` follows
#' `on_error`: "return" (default) returns its message as that partition's value -- the
#' tryCatch contract of README.md:176, 221 --, "restart" fails the gang (a restart), and
#' "raise" stops with the message after the stage.
#' @export
spark_apply <- function(x, f, barrier = TRUE, columns = c(result = "character"), base_port = 8000L,
                        max_restarts = 0L, timeout = 3600, on_error = c("return", "restart", "raise"), ...) {
  stopifnot(inherits(x, "damd_sdf"), isTRUE(barrier))
  on_error <- match.arg(on_error)
  n <- x$partitions
  dir <- tempfile("damd_barrier_")
  dir.create(dir)
  saveRDS(f, file.path(dir, "closure.rds"))
  writeLines(sprintf("127.0.0.1:%d", base_port + seq_len(n) + 100L), file.path(dir, "addresses.txt"))
  runner <- file.path(dir, "runner.R")
  writeLines(c(
    "args <- commandArgs(trailingOnly = TRUE)",
    "dir <- args[1]; mode <- args[2]; i <- as.integer(args[3])",
    "f <- readRDS(file.path(dir, 'closure.rds'))",
    "addr <- readLines(file.path(dir, 'addresses.txt'))",
    "res <- tryCatch(list(ok = TRUE, value = f(data.frame(id = i + 1L), list(address = addr, partition = i))),",
    "                error = function(e) list(ok = FALSE, value = conditionMessage(e)))",
    "saveRDS(res, file.path(dir, sprintf('result-%d.rds', i)))",
    "if (!res$ok && mode == 'restart') quit(save = 'no', status = 3)"
  ), runner)
  launch <- reticulate::import("distributed_amd.launch")
  rscript <- file.path(R.home("bin"), "Rscript")
  gang <- launch$launch_command(c(rscript, runner, dir, on_error), nproc = as.integer(n),
                                max_restarts = as.integer(max_restarts), timeout = timeout, rank_arg = TRUE)
  if (!isTRUE(gang$ok)) {
    stop(sprintf("barrier stage failed after %d attempt(s): worker exit statuses %s", gang$attempts,
                 paste(unlist(gang$returncodes), collapse = ", ")))
  }
  res <- lapply(seq_len(n) - 1L, function(i) readRDS(file.path(dir, sprintf("result-%d.rds", i))))
  if (on_error == "raise") {
    bad <- Filter(function(r) !isTRUE(r$ok), res)
    if (length(bad)) stop(bad[[1]]$value)
  }
  out <- data.frame(vapply(res, function(r) as.character(r$value)[1], character(1)), stringsAsFactors = FALSE)
  names(out) <- names(columns)[1]
  structure(out, class = c("damd_collected", "data.frame"))
}

#' @export
collect <- function(x, ...) {
  class(x) <- "data.frame"
  x
}
