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

#' Gang-scheduled barrier apply: starts one Rscript per partition (all at once), each
#' with barrier = list(address = c(...), partition = i) and DAMD_LOCAL_RANK = i (its
#' GPU), runs `f(df, barrier)` and returns the results in partition order.  A worker
#' error is returned as its message when `f` catches it (README.md:176, 221); a crashed
#' worker fails the whole gang, which is retried up to `max_restarts` times (Spark
#' barrier-stage semantics).
#' @export
spark_apply <- function(x, f, barrier = TRUE, columns = c(result = "character"), base_port = 8000L,
                        max_restarts = 0L, timeout = 3600, ...) {
  stopifnot(inherits(x, "damd_sdf"), isTRUE(barrier))
  n <- x$partitions
  dir <- tempfile("damd_barrier_")
  dir.create(dir)
  fn_file <- file.path(dir, "closure.rds")
  saveRDS(f, fn_file)
  addresses <- sprintf("127.0.0.1:%d", base_port + seq_len(n) + 100L)
  runner <- file.path(dir, "runner.R")
  writeLines(c(
    "args <- commandArgs(trailingOnly = TRUE)",
    "i <- as.integer(args[1]); dir <- args[2]",
    "f <- readRDS(file.path(dir, 'closure.rds'))",
    "addr <- readLines(file.path(dir, 'addresses.txt'))",
    "res <- f(data.frame(id = i + 1L), list(address = addr, partition = i))",
    "saveRDS(res, file.path(dir, sprintf('result-%d.rds', i)))"
  ), runner)
  writeLines(addresses, file.path(dir, "addresses.txt"))
  attempt <- 0L
  repeat {
    pids <- vapply(seq_len(n) - 1L, function(i) {
      env <- c(sprintf("DAMD_LOCAL_RANK=%d", i), sprintf("DAMD_RESTART_COUNT=%d", attempt))
      system2(file.path(R.home("bin"), "Rscript"), c(shQuote(runner), i, shQuote(dir)), wait = FALSE, env = env,
              stdout = file.path(dir, sprintf("worker-%d.log", i)), stderr = file.path(dir, sprintf("worker-%d.log", i)))
      i
    }, integer(1))
    t0 <- Sys.time()
    done <- function() all(file.exists(file.path(dir, sprintf("result-%d.rds", seq_len(n) - 1L))))
    while (!done() && as.numeric(Sys.time() - t0, units = "secs") < timeout) Sys.sleep(0.2)
    if (done()) break
    attempt <- attempt + 1L
    if (attempt > max_restarts) stop("barrier stage failed: not every partition produced a result")
  }
  res <- lapply(seq_len(n) - 1L, function(i) readRDS(file.path(dir, sprintf("result-%d.rds", i))))
  out <- data.frame(vapply(res, function(r) as.character(r)[1], character(1)), stringsAsFactors = FALSE)
  names(out) <- names(columns)[1]
  structure(out, class = c("damd_collected", "data.frame"))
}

#' @export
collect <- function(x, ...) {
  class(x) <- "data.frame"
  x
}
