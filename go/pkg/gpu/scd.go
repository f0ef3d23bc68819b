package gpu

import (
	"context"
	"sync"
	"time"

	"github.com/golang/geo/s2"
	dsserr "github.com/interuss/dss/pkg/errors"
	dssmodels "github.com/interuss/dss/pkg/models"
	scdmodels "github.com/interuss/dss/pkg/scd/models"
	scdstore "github.com/interuss/dss/pkg/scd/store"
)

// SCDTransactor decorates the reference's CockroachDB transactor
// (pkg/scd/store/cockroach, selected in cmds/grpc-backend/main.go): every
// write and point read still goes to CRDB, the source of truth, while
// SearchOperations and SearchSubscriptions run on GPU mirrors of the
// scd_operations / scd_subscriptions 4D columns.  A transaction's writes
// reach the mirrors when it commits; a transaction that has written runs its
// own searches on CRDB, so it sees its own writes exactly as SQL does.
type SCDTransactor struct {
	Inner scdstore.Transactor
	// Now is the store clock (the reference's cockroach.DefaultClock).
	Now func() time.Time

	ops, subs *Mirror
	mu        sync.RWMutex
	opRows    map[scdmodels.ID]*scdmodels.Operation
	subRows   map[scdmodels.ID]*scdmodels.Subscription
}

// NewSCDTransactor builds the mirrors from the tables' current rows (read
// once at start-up, e.g. SELECT * FROM scd_operations / scd_subscriptions).
func NewSCDTransactor(inner scdstore.Transactor, ops []*scdmodels.Operation, subs []*scdmodels.Subscription) (*SCDTransactor, error) {
	t := &SCDTransactor{Inner: inner, Now: time.Now, opRows: map[scdmodels.ID]*scdmodels.Operation{},
		subRows: map[scdmodels.ID]*scdmodels.Subscription{}}
	var err error
	if t.ops, err = NewMirror(false); err != nil {
		return nil, err
	}
	if t.subs, err = NewMirror(true); err != nil {
		return nil, err
	}
	if err := t.apply(ops, nil, subs, nil); err != nil {
		return nil, err
	}
	return t, nil
}

func opRow(o *scdmodels.Operation) Row {
	return Row{Key: o.ID.String(), Cells: o.Cells, AltLo: altOr(o.AltitudeLower, negInf),
		AltHi: altOr(o.AltitudeUpper, posInf), T0: usOrNull(o.StartTime, timeNullStart),
		T1: usOrNull(o.EndTime, timeNullStored), Owner: o.Owner.String()}
}

func subRow(s *scdmodels.Subscription) Row {
	return Row{Key: s.ID.String(), Cells: s.Cells, AltLo: altOr(s.AltitudeLo, negInf),
		AltHi: altOr(s.AltitudeHi, posInf), T0: usOrNull(s.StartTime, timeNullStart),
		T1: usOrNull(s.EndTime, timeNullStored), Owner: s.Owner.String()}
}

// apply writes committed changes to the mirrors and the row caches.
func (t *SCDTransactor) apply(ops []*scdmodels.Operation, delOps []scdmodels.ID, subs []*scdmodels.Subscription, delSubs []scdmodels.ID) error {
	t.mu.Lock()
	defer t.mu.Unlock()
	rows := make([]Row, 0, len(ops))
	for _, o := range ops {
		rows = append(rows, opRow(o))
		t.opRows[o.ID] = o
	}
	if err := t.ops.Upsert(rows); err != nil {
		return err
	}
	keys := make([]string, 0, len(delOps))
	for _, id := range delOps {
		keys = append(keys, id.String())
		delete(t.opRows, id)
	}
	if err := t.ops.Delete(keys); err != nil {
		return err
	}
	rows = rows[:0]
	for _, s := range subs {
		rows = append(rows, subRow(s))
		t.subRows[s.ID] = s
	}
	if err := t.subs.Upsert(rows); err != nil {
		return err
	}
	keys = keys[:0]
	for _, id := range delSubs {
		keys = append(keys, id.String())
		delete(t.subRows, id)
	}
	return t.subs.Delete(keys)
}

// Transact implements scdstore.Transactor.
func (t *SCDTransactor) Transact() (scdstore.Transaction, error) {
	tx, err := t.Inner.Transact()
	if err != nil {
		return nil, err
	}
	return &scdTx{inner: tx, t: t, ops: map[scdmodels.ID]*scdmodels.Operation{},
		subs: map[scdmodels.ID]*scdmodels.Subscription{}}, nil
}

// scdTx records a transaction's writes (nil value: deleted) until commit.
type scdTx struct {
	inner scdstore.Transaction
	t     *SCDTransactor
	ops   map[scdmodels.ID]*scdmodels.Operation
	subs  map[scdmodels.ID]*scdmodels.Subscription
}

func (x *scdTx) Store() (scdstore.Store, error) {
	s, err := x.inner.Store()
	if err != nil {
		return nil, err
	}
	return &scdStore{Store: s, tx: x}, nil
}

func (x *scdTx) Commit() error {
	if err := x.inner.Commit(); err != nil {
		return err
	}
	return x.flush()
}

func (x *scdTx) flush() error {
	var ups []*scdmodels.Operation
	var dels []scdmodels.ID
	for id, o := range x.ops {
		if o == nil {
			dels = append(dels, id)
		} else {
			ups = append(ups, o)
		}
	}
	var sups []*scdmodels.Subscription
	var sdels []scdmodels.ID
	for id, s := range x.subs {
		if s == nil {
			sdels = append(sdels, id)
		} else {
			sups = append(sups, s)
		}
	}
	x.ops, x.subs = map[scdmodels.ID]*scdmodels.Operation{}, map[scdmodels.ID]*scdmodels.Subscription{}
	return x.t.apply(ups, dels, sups, sdels)
}

func (x *scdTx) Rollback() error {
	x.ops, x.subs = map[scdmodels.ID]*scdmodels.Operation{}, map[scdmodels.ID]*scdmodels.Subscription{}
	return x.inner.Rollback()
}

func (x *scdTx) dirty() bool { return len(x.ops) > 0 || len(x.subs) > 0 }

// scdStore is the store a transaction hands out: the CRDB store with the
// searches replaced.
type scdStore struct {
	scdstore.Store
	tx *scdTx
}

// refreshSub re-reads a subscription a write may have created or removed
// (the implicit subscription of UpsertOperation / DeleteOperation,
// operations.go:239-372).
func (s *scdStore) refreshSub(ctx context.Context, id scdmodels.ID, owner dssmodels.Owner) {
	if id.Empty() {
		return
	}
	sub, err := s.Store.GetSubscription(ctx, id, owner)
	if err == nil && sub != nil {
		s.tx.subs[id] = sub
	} else {
		s.tx.subs[id] = nil
	}
}

func (s *scdStore) UpsertOperation(ctx context.Context, op *scdmodels.Operation, key []scdmodels.OVN) (*scdmodels.Operation, []*scdmodels.Subscription, error) {
	res, subs, err := s.Store.UpsertOperation(ctx, op, key)
	if err == nil && res != nil {
		s.tx.ops[res.ID] = res
		s.refreshSub(ctx, res.SubscriptionID, res.Owner)
	}
	return res, subs, err
}

func (s *scdStore) DeleteOperation(ctx context.Context, id scdmodels.ID, owner dssmodels.Owner) (*scdmodels.Operation, []*scdmodels.Subscription, error) {
	res, subs, err := s.Store.DeleteOperation(ctx, id, owner)
	if err == nil {
		s.tx.ops[id] = nil
		if res != nil {
			s.refreshSub(ctx, res.SubscriptionID, owner)
		}
	}
	return res, subs, err
}

func (s *scdStore) UpsertSubscription(ctx context.Context, sub *scdmodels.Subscription) (*scdmodels.Subscription, []*scdmodels.Operation, error) {
	res, ops, err := s.Store.UpsertSubscription(ctx, sub)
	if err == nil && res != nil {
		s.tx.subs[res.ID] = res
	}
	return res, ops, err
}

func (s *scdStore) DeleteSubscription(ctx context.Context, id scdmodels.ID, owner dssmodels.Owner, version scdmodels.Version) (*scdmodels.Subscription, error) {
	res, err := s.Store.DeleteSubscription(ctx, id, owner, version)
	if err == nil {
		s.tx.subs[id] = nil
	}
	return res, err
}

// SearchOperations replaces searchOperations
// (pkg/scd/store/cockroach/operations.go:374-435): the same argument checks
// and error messages, then
//   cells && cells AND COALESCE(altitude_upper >= lo, true)
//   AND COALESCE(altitude_lower <= hi, true) AND COALESCE(ends_at >= start, true)
//   AND COALESCE(starts_at <= end, true) AND ends_at >= now
// on the GPU mirror.  The owner argument is unused, as in the reference.
func (s *scdStore) SearchOperations(ctx context.Context, v4d *dssmodels.Volume4D, owner dssmodels.Owner) ([]*scdmodels.Operation, error) {
	if s.tx.dirty() {
		return s.Store.SearchOperations(ctx, v4d, owner)
	}
	if v4d.SpatialVolume == nil || v4d.SpatialVolume.Footprint == nil {
		return nil, dsserr.BadRequest("missing geospatial footprint for query")
	}
	cells, err := Geometry(v4d.SpatialVolume.Footprint).CalculateCovering()
	if err != nil {
		return nil, dsserr.BadRequest(err.Error())
	}
	if len(cells) == 0 {
		return nil, dsserr.BadRequest("missing cell IDs for query")
	}
	t := s.tx.t
	now := t.Now().UnixNano() / 1000
	tlo := now // ends_at >= now, and ends_at >= start when start is set
	if v4d.StartTime != nil {
		if st := v4d.StartTime.UnixNano() / 1000; st > tlo {
			tlo = st
		}
	}
	q := Query{Cells: cells, AltLo: altOr(v4d.SpatialVolume.AltitudeLo, negInf),
		AltHi: altOr(v4d.SpatialVolume.AltitudeHi, posInf), TLo: tlo, THi: usOrNull(v4d.EndTime, timeNullEndQ)}
	keys, err := t.ops.Search([]Query{q})
	if err != nil {
		return nil, err
	}
	t.mu.RLock()
	defer t.mu.RUnlock()
	out := make([]*scdmodels.Operation, 0, len(keys[0]))
	for _, k := range keys[0] {
		if o, ok := t.opRows[scdmodels.ID(k)]; ok {
			c := *o
			out = append(out, &c)
		}
	}
	return out, nil
}

// SearchSubscriptions replaces the SCD SubscriptionStore.SearchSubscriptions
// (pkg/scd/store/cockroach/subscriptions.go:497-545).  Its LEFT JOIN keeps
// every row of the owner, so the cells only have to be non-empty (quirk Q7):
// the answer is the owner's subscriptions with ends_at >= now.
func (s *scdStore) SearchSubscriptions(ctx context.Context, cells s2.CellUnion, owner dssmodels.Owner) ([]*scdmodels.Subscription, error) {
	if s.tx.dirty() {
		return s.Store.SearchSubscriptions(ctx, cells, owner)
	}
	if len(cells) == 0 {
		return nil, dsserr.BadRequest("no location provided")
	}
	t := s.tx.t
	now := t.Now()
	t.mu.RLock()
	defer t.mu.RUnlock()
	var out []*scdmodels.Subscription
	for _, sub := range t.subRows {
		if sub.Owner == owner && sub.EndTime != nil && !sub.EndTime.Before(now) {
			c := *sub
			out = append(out, &c)
		}
	}
	return out, nil
}
