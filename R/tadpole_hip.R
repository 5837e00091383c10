# Copyright (C) the TADpole authors (3DGenomes/TADpole, GPL-3) and the
# tadpole_amd authors.
#
# This file is part of a GPU backend for the TADpole R package.  Parts of it
# restate the reference's R code (R/TADpole.R) so that TADpole_hip() is a
# drop-in for TADpole(); like the reference (DESCRIPTION: License GPL-3) it is
# free software: you can redistribute it and/or modify it under the terms of
# the GNU General Public License as published by the Free Software Foundation,
# either version 3 of the License, or (at your option) any later version.
# It is distributed WITHOUT ANY WARRANTY; without even the implied warranty of
# MERCHANTABILITY or FITNESS FOR A PARTICULAR PURPOSE.  See the GNU General
# Public License (https://www.gnu.org/licenses/gpl-3.0.html) for details.
#
# tadpole_hip.R -- R host side of libtadpole_hip.so (the MI355X engine) for the
# 3DGenomes/TADpole package.  Drop this file into the package's R/ directory:
# TADpole_hip() is TADpole() (R/TADpole.R:344-501) with the hot path -- mask,
# sparse_cor, prcomp, find_params and the final chclust (R/TADpole.R:444-460,
# 362-374) -- running on the GPU through the pointer-only C ABI of
# include/tadpole_hip.h (`.C`, no R headers).  The assembly of the `tadpole`
# object, fix_values (R/TADpole.R:503-510), the centromere split and the arm
# merge stay the reference's R code.  R is not installed in the build image, so
# this file is not exercised by the repository's tests; the Python mirror
# (tadpole_amd/api.py) runs the same C ABI in tests/.

.tp_lib <- function() {
  if (!is.loaded("tp_pipeline"))
    dyn.load(Sys.getenv("TADPOLE_HIP_LIB", "libtadpole_hip.so"))
  invisible(TRUE)
}

.tp_error <- function(status) {
  msg <- .C("tp_last_error_r", msg = strrep(" ", 1024L), len = 1024L)$msg
  stop(sprintf("libtadpole_hip status %d: %s", status, trimws(msg)), call. = FALSE)
}

TP_FLAG_CLEAN <- 2L     # input already NA-free and symmetric
TP_FLAG_NO_MASK <- 4L   # keep every bin (the per-arm matrices of R/TADpole.R:362)

# read.big.matrix(mat_file, type = 'double', sep = '\t') (R/TADpole.R:17): a
# memory-mapped, multi-threaded native parse; NA fields arrive as NaN.
read_matrix_hip <- function(mat_file, nthreads = 0L) {
  .tp_lib()
  d <- .C("tp_tsv_dims", path = as.character(mat_file), nrow = integer(1), ncol = integer(1),
          status = integer(1))
  if (d$status != 0L) .tp_error(d$status)
  r <- .C("tp_read_tsv", path = as.character(mat_file), nrow = d$nrow, ncol = d$ncol,
          nthreads = as.integer(nthreads), flags = 0L,      # 0 = column-major, R's layout
          out = double(d$nrow * d$ncol), status = integer(1), NAOK = TRUE)
  if (r$status != 0L) .tp_error(r$status)
  matrix(r$out, nrow = d$nrow, ncol = d$ncol)
}

# One tp_pipeline call: NA->0 + forceSymmetric(uplo='U') + mask (unless
# TP_FLAG_NO_MASK) + cor + prcomp + find_params + the tree of n_PCs.
.tp_pipeline <- function(mat, max_pcs, min_clusters, bad_frac, flags = 0L, device = 0L) {
  .tp_lib()
  storage.mode(mat) <- "double"
  n0 <- nrow(mat); k_cap <- min(max_pcs, n0); w_cap <- n0
  r <- .C("tp_pipeline",
          M = mat, n0 = as.integer(n0), max_pcs = as.integer(max_pcs),
          min_clusters = as.integer(min_clusters), bad_frac = as.double(bad_frac),
          flags = as.integer(flags), device = as.integer(device),
          k_cap = as.integer(k_cap), w_cap = as.integer(w_cap),
          bad = integer(n0), n_good = integer(1), good_idx = integer(n0),
          k = integer(1), n_cluster = integer(k_cap), scores = double(k_cap * w_cap),
          w = integer(1), n_pcs = integer(1), n_clusters = integer(1),
          merge = integer(2 * max(1, n0 - 1)), height = double(max(1, n0 - 1)),
          boundary = integer(max(1, n0 - 1)), timings = double(32), status = integer(1),
          NAOK = TRUE)
  if (r$status != 0L) .tp_error(r$status)
  r
}

# The `tadpole` list of R/TADpole.R:463-497 from a pipeline result; `labels`:
# the row names of the clustered matrix (original bin indices), `bad_columns`
# as the reference keeps them.  The per-level loop is the reference's code.
.tp_assemble <- function(r, labels, bad_columns, slot = "clusters") {
  n <- r$n_good; k <- r$k; w <- r$w
  scores <- matrix(r$scores[seq_len(k * w)], nrow = k, ncol = w, dimnames = list(1:k, 1:w))
  dendro <- structure(list(merge = matrix(r$merge[seq_len(2 * (n - 1))], ncol = 2),
                           height = r$height[seq_len(n - 1)], order = seq_len(n),
                           labels = as.character(labels), method = "coniss",
                           call = quote(rioja::chclust(d = dist(pcs))), dist.method = "euclidean"),
                      class = c("chclust", "hclust"))
  out <- list(n_pcs = r$n_pcs, optimal_n_clusters = r$n_clusters, dendro = dendro)
  out[[slot]] <- list()
  for (kk in which(!is.na(scores[r$n_pcs, ]))) {
    good_clusters <- cutree(dendro, k = kk)
    if (!is.null(bad_columns)) {
      bad_clusters <- rep(0, length(bad_columns)); names(bad_clusters) <- bad_columns
      clusters <- c(good_clusters, bad_clusters)
      clusters <- clusters[order(as.numeric(names(clusters)))]
      fixed <- inverse.rle(fix_values(rle(clusters)))
      eb <- cumsum(rle(fixed)$length)
      coord <- data.frame(start = c(1, eb[-length(eb)] + 1, use.names = FALSE), end = eb)
      coord <- coord[rle(fixed)$values != 0, ]
    } else {
      eb <- cumsum(table(good_clusters))
      coord <- data.frame(start = c(1, eb[-length(eb)] + 1, use.names = FALSE), end = eb)
    }
    out[[slot]][[as.character(kk)]] <- coord
  }
  if (slot == "clusters") out$scores <- scores
  out
}

# TADpole() (R/TADpole.R:344-501) on the GPU.  `mat_file`: a path (native
# reader) or an in-memory matrix.  Plots of load_mat are not drawn.
# Limit: min(max_pcs, number of good bins) <= 1024 -- the sweep's kernels hold
# at most 1024 PC columns per tree (16 column slots of 64) and the PCA's own
# eigensolver blocks up to 1280; R itself has no cap (R/TADpole.R:344,452).
# Larger values stop with the library's TP_ERR_UNSUPPORTED message.
TADpole_hip <- function(mat_file, max_pcs = 200, min_clusters = 2, bad_frac = 0.01,
                        chr, start, end, resol, centromere_search = FALSE, device = 0L) {
  if (max_pcs > 1024) {
    nb <- if (is.character(mat_file)) NA else nrow(as.matrix(mat_file))
    if (is.na(nb) || nb > 1024)
      warning("max_pcs > 1024: supported only while the matrix keeps <= 1024 good bins (sweep limit)")
  }
  mat <- if (is.character(mat_file)) read_matrix_hip(mat_file) else as.matrix(mat_file)
  if (!centromere_search) {
    r <- .tp_pipeline(mat, max_pcs, min_clusters, bad_frac, 0L, device)
    bad_columns <- as.character(which(r$bad != 0L))
    message(paste(length(bad_columns), 'bad columns found at position(s):'))
    message(paste(bad_columns, collapse = ' '))
    good <- r$good_idx[seq_len(r$n_good)]
    message(paste('Optimal number of PCs:', r$n_pcs))
    message(paste('Optimal number of clusters:', r$n_clusters))
    return(structure(.tp_assemble(r, good, bad_columns), class = 'tadpole'))
  }
  # load_mat's centromere split (R/TADpole.R:19-20,35-37,58-85), the reference's
  # own code (bug-compatible: q-arm bad bins removed by original index, :78-80)
  mat[is.na(mat)] <- 0
  mat <- as.matrix(Matrix::forceSymmetric(mat, uplo = 'U'))
  rownames(mat) <- 1:nrow(mat); colnames(mat) <- 1:ncol(mat)
  r <- rowMeans(mat)
  bad <- diag(mat) == 0
  if (bad_frac) bad <- bad | r < quantile(r, seq(0, 1, by = bad_frac))[2]
  message(paste(sum(bad), 'bad columns found at position(s):'))
  message(paste(names(which(bad)), collapse = ' '))
  if (!any(bad)) stop("$ operator is invalid for atomic vectors")     # R/TADpole.R:87-90,356
  idx <- as.numeric(names(which(bad)))
  runs <- split(idx, cumsum(seq_along(idx) %in% (which(diff(idx) > 1) + 1)))
  cs <- head(runs[[which.max(lengths(runs))]], 1); ce <- tail(runs[[which.max(lengths(runs))]], 1)
  message(paste('centromere position:', cs, ce))
  if (cs == 1 || ce == nrow(mat)) {                                   # :66-70, then :356
    message('longest stretch of bad rows/columns at the ends, not splitting the matrix.')
    stop("$ operator is invalid for atomic vectors")
  }
  arms <- list(p = mat[1:(cs - 1), 1:(cs - 1)], q = mat[(ce + 1):nrow(mat), (ce + 1):nrow(mat)])
  bads <- list(p = idx[idx < cs], q = idx[idx > ce])
  if (length(bads$p)) arms$p <- arms$p[-bads$p, -bads$p]
  if (length(bads$q)) arms$q <- arms$q[-bads$q, -bads$q]
  centromer <- cs:ce
  tadpole <- structure(list(), class = 'tadpole')
  fixed_clusters_arms <- c()
  for (arm in c('p', 'q')) {
    message(paste('Processing arm', arm))
    m <- arms[[arm]]
    r <- .tp_pipeline(m, max_pcs, min_clusters, 0, TP_FLAG_CLEAN + TP_FLAG_NO_MASK, device)
    message(paste('Optimal number of PCs:', r$n_pcs))
    message(paste('Optimal number of clusters:', r$n_clusters))
    t <- .tp_assemble(r, rownames(m), bads[[arm]], slot = 'cluster')   # `$cluster`, R/TADpole.R:407
    tadpole[[arm]] <- t
    good_clusters <- cutree(t$dendro, k = r$n_clusters)
    bad_clusters <- rep(0, length(bads[[arm]])); names(bad_clusters) <- bads[[arm]]
    clusters <- c(good_clusters, bad_clusters)
    clusters <- clusters[order(as.numeric(names(clusters)))]
    fixed_clusters_arms <- c(fixed_clusters_arms, inverse.rle(fix_values(rle(clusters))),
                             rep(0, length(centromer)))
  }
  v <- fixed_clusters_arms[1:(length(fixed_clusters_arms) - length(centromer))]
  eb <- cumsum(rle(v)$lengths)
  coord <- data.frame(start = c(1, eb[-length(eb)] + 1, use.names = TRUE), end = eb)
  tadpole$merging_arms <- coord[rle(v)$values != 0, ]
  tadpole
}

# stats::dist(pcs) (R/TADpole.R:108,460) in R's accumulation order.
dist_hip <- function(pcs, device = 0L) {
  .tp_lib(); n <- nrow(pcs)
  r <- .C("tp_dist", P = as.double(pcs), n = as.integer(n), ncols = as.integer(ncol(pcs)),
          device = as.integer(device), d = double(n * (n - 1) / 2), status = integer(1))
  if (r$status != 0L) .tp_error(r$status)
  structure(r$d, Size = n, Labels = rownames(pcs), Diag = FALSE, Upper = FALSE,
            method = "euclidean", class = "dist")
}
