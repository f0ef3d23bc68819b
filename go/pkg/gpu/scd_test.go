package gpu

// Needs cgo, libdss_amd.so and a gfx950 device; not compiled in the image
// this was written in (no Go toolchain: INTEGRATION.md "Status").  The same
// protocol is replayed from C in tests/host/abi_test.c.

import (
	"context"
	"sync"
	"testing"
	"time"

	"github.com/golang/geo/s2"
	dssmodels "github.com/interuss/dss/pkg/models"
	scderr "github.com/interuss/dss/pkg/scd/errors"
	scdmodels "github.com/interuss/dss/pkg/scd/models"
	scdstore "github.com/interuss/dss/pkg/scd/store"
	scdc "github.com/interuss/dss/pkg/scd/store/cockroach"
	"google.golang.org/grpc/codes"
	"google.golang.org/grpc/status"
)

// fakeDB stands in for CockroachDB: committed operations, and a store per
// transaction whose UpsertOperation runs the reference's OVN check over the
// installed ConflictSearch hook (operations.go:333-360) and records the row.
type fakeDB struct {
	mu   sync.Mutex
	ops  map[scdmodels.ID]*scdmodels.Operation
	subs map[scdmodels.ID]*scdmodels.Subscription
}

type fakeTx struct {
	db          *fakeDB
	pending     []*scdmodels.Operation
	pendingSubs []*scdmodels.Subscription
}

type fakeStore struct {
	scdstore.Store // the methods the test does not call
	tx             *fakeTx
	hooks          *scdc.Hooks
}

func (s *fakeStore) SetHooks(h *scdc.Hooks) { s.hooks = h }

func (s *fakeStore) UpsertOperation(ctx context.Context, op *scdmodels.Operation, key []scdmodels.OVN) (*scdmodels.Operation, []*scdmodels.Subscription, error) {
	found, err := s.hooks.ConflictSearch(ctx, op)
	if err != nil {
		return nil, nil, err
	}
	have := map[scdmodels.OVN]bool{}
	for _, k := range key {
		have[k] = true
	}
	for _, o := range found {
		if !have[o.OVN] {
			return nil, nil, scderr.MissingOVNsInternalError()
		}
	}
	time.Sleep(20 * time.Millisecond) // widen the window between the check and the commit
	s.tx.pending = append(s.tx.pending, op)
	// pushOperation's fan-out (operations.go:186 -> subscriptions.go:128-173)
	var subs []*scdmodels.Subscription
	if s.hooks.NotificationSearch != nil {
		cells := make([]int64, len(op.Cells))
		for i, c := range op.Cells {
			cells[i] = int64(c)
		}
		ids, err := s.hooks.NotificationSearch(ctx, cells)
		if err != nil {
			return nil, nil, err
		}
		for _, id := range ids {
			subs = append(subs, &scdmodels.Subscription{ID: id})
		}
	}
	return op, subs, nil
}

// UpsertSubscription: the reference's SQL search of the operations its area
// covers (subscriptions.go:416), over what CRDB has committed, then the row.
func (s *fakeStore) UpsertSubscription(ctx context.Context, sub *scdmodels.Subscription) (*scdmodels.Subscription, []*scdmodels.Operation, error) {
	time.Sleep(20 * time.Millisecond)
	s.tx.db.mu.Lock()
	var ops []*scdmodels.Operation
	for _, o := range s.tx.db.ops {
		for _, c := range o.Cells {
			if sub.Cells.ContainsCellID(c) {
				ops = append(ops, o)
				break
			}
		}
	}
	s.tx.db.mu.Unlock()
	s.tx.pendingSubs = append(s.tx.pendingSubs, sub)
	return sub, ops, nil
}

func (s *fakeStore) GetSubscription(ctx context.Context, id scdmodels.ID, owner dssmodels.Owner) (*scdmodels.Subscription, error) {
	return nil, nil
}

func (x *fakeTx) Store() (scdstore.Store, error) { return &fakeStore{tx: x}, nil }

func (x *fakeTx) Commit() error {
	x.db.mu.Lock()
	defer x.db.mu.Unlock()
	for _, o := range x.pending {
		x.db.ops[o.ID] = o
	}
	for _, sub := range x.pendingSubs {
		x.db.subs[sub.ID] = sub
	}
	return nil
}

func (x *fakeTx) Rollback() error { return nil }

func (db *fakeDB) Transact() (scdstore.Transaction, error) { return &fakeTx{db: db}, nil }

// Two concurrent upserts of overlapping Accepted operations with empty keys:
// in the reference CRDB's SERIALIZABLE isolation lets only one commit; the
// mirror path must do the same (ADVICE r3: write skew), so exactly one gets
// MissingOVNs.
func TestConcurrentOverlappingUpsertsOneMissingOVNs(t *testing.T) {
	tr, err := NewSCDTransactor(newFakeDB(), nil, nil)
	if err != nil {
		t.Skipf("no GPU mirror: %v", err)
	}
	start, end := time.Now(), time.Now().Add(time.Hour)
	lo, hi := float32(0), float32(100)
	cell := s2.CellIDFromToken("808fb0ac")
	mk := func(id string) *scdmodels.Operation {
		return &scdmodels.Operation{ID: scdmodels.ID(id), Owner: "uss", State: scdmodels.OperationStateAccepted,
			Cells: s2.CellUnion{cell}, StartTime: &start, EndTime: &end, AltitudeLower: &lo, AltitudeUpper: &hi,
			OVN: scdmodels.OVN(id)}
	}
	ids := []string{"00000000-0000-4000-8000-000000000001", "00000000-0000-4000-8000-000000000002"}
	errs := make([]error, 2)
	var wg sync.WaitGroup
	for i := range ids {
		wg.Add(1)
		go func(i int) {
			defer wg.Done()
			errs[i] = scdstore.PerformOperationWithRetries(context.Background(), tr,
				func(ctx context.Context, st scdstore.Store) error {
					_, _, err := st.UpsertOperation(ctx, mk(ids[i]), nil)
					return err
				}, 0)
		}(i)
	}
	wg.Wait()
	missing := 0
	for _, e := range errs {
		if e == scderr.MissingOVNsInternalError() {
			missing++
		} else if e != nil {
			t.Fatalf("unexpected error %v", e)
		}
	}
	if missing != 1 {
		t.Fatalf("want exactly one MissingOVNs, got %d (%v)", missing, errs)
	}
}

// An empty covering is rejected as searchOperations does
// (operations.go:405-414), before the mirror is searched.
func TestConflictSearchEmptyCells(t *testing.T) {
	tr, err := NewSCDTransactor(newFakeDB(), nil, nil)
	if err != nil {
		t.Skipf("no GPU mirror: %v", err)
	}
	x, _ := tr.Transact()
	st, _ := x.Store()
	_, err = st.(*scdStore).conflicts(context.Background(), &scdmodels.Operation{})
	if st, ok := status.FromError(err); err == nil || !ok || st.Code() != codes.InvalidArgument ||
		st.Message() != "missing cell IDs for query" {
		t.Fatalf("want BadRequest(missing cell IDs for query), got %v", err)
	}
	_ = x.Rollback()
}

func newFakeDB() *fakeDB {
	return &fakeDB{ops: map[scdmodels.ID]*scdmodels.Operation{}, subs: map[scdmodels.ID]*scdmodels.Subscription{}}
}

// An operation upsert and a subscription upsert over the same cell, run
// concurrently: in the reference CRDB's SERIALIZABLE isolation orders them,
// so either the operation's notification fan-out names the subscription or
// the subscription's operation search returns the operation (ADVICE r4: the
// fan-out reads the mirror, so both must run under the write lock).
func TestConcurrentOperationAndSubscriptionSeeEachOther(t *testing.T) {
	for rep := 0; rep < 20; rep++ {
		tr, err := NewSCDTransactor(newFakeDB(), nil, nil)
		if err != nil {
			t.Skipf("no GPU mirror: %v", err)
		}
		start, end := time.Now(), time.Now().Add(time.Hour)
		lo, hi := float32(0), float32(100)
		cell := s2.CellIDFromToken("808fb0ac")
		op := &scdmodels.Operation{ID: "00000000-0000-4000-8000-000000000011", Owner: "uss",
			State: scdmodels.OperationStateAccepted, Cells: s2.CellUnion{cell}, StartTime: &start, EndTime: &end,
			AltitudeLower: &lo, AltitudeUpper: &hi, OVN: "ovn"}
		sub := &scdmodels.Subscription{ID: "00000000-0000-4000-8000-000000000012", Owner: "uss2",
			Cells: s2.CellUnion{cell}, StartTime: &start, EndTime: &end, AltitudeLo: &lo, AltitudeHi: &hi}
		var notified []*scdmodels.Subscription
		var seen []*scdmodels.Operation
		var wg sync.WaitGroup
		wg.Add(2)
		go func() {
			defer wg.Done()
			_ = scdstore.PerformOperationWithRetries(context.Background(), tr,
				func(ctx context.Context, st scdstore.Store) error {
					var err error
					_, notified, err = st.UpsertOperation(ctx, op, nil)
					return err
				}, 0)
		}()
		go func() {
			defer wg.Done()
			_ = scdstore.PerformOperationWithRetries(context.Background(), tr,
				func(ctx context.Context, st scdstore.Store) error {
					var err error
					_, seen, err = st.UpsertSubscription(ctx, sub)
					return err
				}, 0)
		}()
		wg.Wait()
		if len(notified) == 0 && len(seen) == 0 {
			t.Fatalf("rep %d: neither the operation's fan-out nor the subscription's search saw the other", rep)
		}
	}
}
