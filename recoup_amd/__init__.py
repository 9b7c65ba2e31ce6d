"""recoup_amd -- MI355X-native engine for recoup's coverage -> profile hot path.

Mirrors the reference's R API for that path (hjanime/recoup R/coverage.R, R/profile.R):
``calcCoverage``, ``coverageRef``, ``coverageRnaRef``, ``profileMatrix`` and the internal
``binCoverageMatrix`` / ``baseCoverageMatrix``, computed by hand-written gfx950 HIP kernels
behind the C ABI in ``include/recoup_amd.h``.
"""
__version__ = "0.1.0"

from .granges import (GRanges, GRangesList, flank, getFlankingRanges, getRegionalRanges,  # noqa: F401
                      promoters, resize)
from .api import (CoverageList, DeviceCoverage, RMatrix, Rle, baseCoverageMatrix, binCoverageMatrix,  # noqa: F401
                  calcCoverage, calcLinearFactors, coverageRef, coverageRnaRef, normalizeLinear, profileMatrix,
                  RRng, preprocessRanges, readBam, recoupProfiles)
from ._lib import RcpError, SemanticError, UnsupportedError  # noqa: F401
