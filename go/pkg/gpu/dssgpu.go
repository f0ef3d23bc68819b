// Package gpu binds libdss_amd.so (include/dssgpu.h) to the reference's Go
// interfaces: the covering behind models.Geometry / geo.Covering /
// geo.AreaToCellIDs, and GPU-resident search mirrors behind
// scdstore.OperationStore, scdstore.SubscriptionStore, repos.ISA and
// repos.Subscription (see INTEGRATION.md for where a maintainer selects them).
//
// Build: copy include/dssgpu.h and libdss_amd.so into
// third_party/dssgpu/{include,lib} of the reference checkout, drop this
// directory in as pkg/gpu, and apply go/patches/0001-export-geo-errors.patch
// (two added files: the sentinel errors and the ErrAreaTooLarge constructor
// the covering needs to return byte-identical errors).
//
// No Go toolchain exists in the image this was written in: the package is
// source only; the same ABI is exercised from C (tests/host/abi_test.c) and
// from Python (dss_amd/_lib.py) by the test suite.
package gpu

/*
#cgo CFLAGS: -I${SRCDIR}/../../third_party/dssgpu/include
#cgo LDFLAGS: -L${SRCDIR}/../../third_party/dssgpu/lib -ldss_amd -Wl,-rpath,${SRCDIR}/../../third_party/dssgpu/lib
#include <stdlib.h>
#include "dssgpu.h"
*/
import "C"

import (
	"fmt"
	"math"
	"sync"
	"time"
	"unsafe"

	"github.com/golang/geo/s2"
)

// Device is the GPU ordinal every context of this process opens (one
// process per GPU: set it before the first call, e.g. from LOCAL_RANK).
var Device = 0

// ctx is one engine context: a HIP stream plus the engines' scratch.  The C
// ABI is re-entrant across contexts, so calls draw a context from a pool and
// concurrent RPC goroutines run on independent contexts.
type ctx struct{ c *C.dssg_ctx }

var (
	poolMu  sync.Mutex
	pool    []*ctx
	initErr error
)

func getCtx() (*ctx, error) {
	poolMu.Lock()
	if n := len(pool); n > 0 {
		c := pool[n-1]
		pool = pool[:n-1]
		poolMu.Unlock()
		return c, nil
	}
	poolMu.Unlock()
	var c *C.dssg_ctx
	if rc := C.dssg_create(C.int(Device), &c); rc != C.DSSG_OK {
		return nil, fmt.Errorf("dssg_create: %s", C.GoString(C.dssg_strerror(rc)))
	}
	return &ctx{c}, nil
}

func putCtx(c *ctx) {
	poolMu.Lock()
	pool = append(pool, c)
	poolMu.Unlock()
}

func (c *ctx) err(call string, rc C.int) error {
	msg := C.GoString(C.dssg_last_error(c.c))
	if msg == "" {
		msg = C.GoString(C.dssg_strerror(rc))
	}
	return fmt.Errorf("%s: %s", call, msg)
}

// ---- times and altitudes (the ABI's NULL sentinels, dssgpu.h) ------------

const (
	timeNullStart  = math.MinInt64 // DSSG_TIME_NULL_START
	timeNullEndQ   = math.MaxInt64 // DSSG_TIME_NULL_END_Q: a query end that is NULL
	timeNullStored = math.MinInt64 // DSSG_TIME_NULL_END: a stored ends_at NULL never matches
)

// usOf is a time as CockroachDB stores and compares a TIMESTAMPTZ: rounded
// to the microsecond (tree.MakeDTimestampTZ rounds with time.Round, half
// up), as int64 microseconds since the Unix epoch.  Every time that reaches
// the mirrors -- query bounds, now, stored rows -- goes through it, so a
// bound within 500 ns of a stored value compares as it does in SQL.
func usOf(t time.Time) int64 {
	return t.Round(time.Microsecond).UnixNano() / 1000
}

func usOrNull(t *time.Time, null int64) int64 {
	if t == nil {
		return null
	}
	return usOf(*t)
}

func altOr(a *float32, null float32) float32 {
	if a == nil {
		return null
	}
	return *a
}

var (
	negInf = float32(math.Inf(-1))
	posInf = float32(math.Inf(1))
)

// ---- cell lists -----------------------------------------------------------

func cellsPtr(cu s2.CellUnion) *C.uint64_t {
	if len(cu) == 0 {
		return nil
	}
	return (*C.uint64_t)(unsafe.Pointer(&cu[0]))
}

func toCellUnion(cells []uint64) s2.CellUnion {
	cu := make(s2.CellUnion, len(cells))
	for i, c := range cells {
		cu[i] = s2.CellID(c)
	}
	return cu
}
