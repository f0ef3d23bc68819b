package gpu

import (
	"context"
	"sync"
	"sync/atomic"
	"time"

	"github.com/golang/geo/s2"
	dsserr "github.com/interuss/dss/pkg/errors"
	dssmodels "github.com/interuss/dss/pkg/models"
	scdmodels "github.com/interuss/dss/pkg/scd/models"
	scdstore "github.com/interuss/dss/pkg/scd/store"
	scdc "github.com/interuss/dss/pkg/scd/store/cockroach"
)

// SCDTransactor decorates the reference's CockroachDB transactor
// (pkg/scd/store/cockroach, selected in cmds/grpc-backend/main.go).  CRDB
// stays the source of truth for every row write and point read; the 4D
// searches run on GPU mirrors of the scd_operations / scd_subscriptions
// columns:
//   - SearchOperations and SearchSubscriptions;
//   - through the store hooks of go/patches/0002 (Store.SetHooks), the write
//     path's two searches: UpsertOperation's conflict search
//     (operations.go:337-348; the OVN check itself stays the reference's) and
//     the notification fan-out's subscription ids
//     (fetchSubscriptionsForNotification, subscriptions.go:128-173; CRDB runs
//     only the UPDATE ... RETURNING of their counters);
//   - inside a transaction, the searches see its own uncommitted writes
//     (read-your-writes): the mirror's answer minus the rows the transaction
//     has written, plus those of its written rows that match.
// A transaction's writes reach the mirrors when it commits.
//
// Serialisation of the write path.  In the reference the conflict search and
// the notification fan-out are SQL reads inside SERIALIZABLE transactions, so
// CRDB aborts one of two concurrent transactions whose reads and writes
// overlap: of an operation upsert and a subscription upsert that cover the
// same cells, either the operation's fan-out sees the subscription or the
// subscription's own operation search (subscriptions.go:416) sees the
// operation.  A mirror read registers nothing with CRDB, so every writing
// transaction takes the transactor's write lock before its first write or
// write-path mirror search (conflict search, notification fan-out) and holds
// it until its commit has been applied to the mirrors (or it rolls back):
// writers run one at a time, each seeing every earlier writer's rows.  No
// writer waits for the lock while holding CRDB write intents (it takes the
// lock before its first write), so the lock cannot deadlock against CRDB's
// own locks.  Read-only searches do not take it.  The mirrors see only this
// process's writes (single writer per CRDB cluster, INTEGRATION.md); if
// applying a committed transaction to them fails, they are marked invalid
// and every search goes to CRDB from then on.
type SCDTransactor struct {
	Inner scdstore.Transactor
	// Now is the store clock (the reference's cockroach.DefaultClock).
	Now func() time.Time

	ops, subs *Mirror
	mu        sync.RWMutex
	writeMu   sync.Mutex // held by a writing transaction from its first write / write-path search to its commit's apply
	opRows    map[scdmodels.ID]*scdmodels.Operation
	subRows   map[scdmodels.ID]*scdmodels.Subscription
	invalid   int32 // atomic: 1 after a failed apply of a committed transaction
}

// Invalid reports whether the mirrors fell behind CRDB (searches then run on CRDB).
func (t *SCDTransactor) Invalid() bool { return atomic.LoadInt32(&t.invalid) != 0 }

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
	inner  scdstore.Transaction
	t      *SCDTransactor
	ops    map[scdmodels.ID]*scdmodels.Operation
	subs   map[scdmodels.ID]*scdmodels.Subscription
	locked bool // holds t.writeMu (it wrote, or ran a write-path search)
}

// hookable is the reference store with the hooks of
// go/patches/0002-scd-rid-gpu-store-hooks.patch.
type hookable interface {
	SetHooks(h *scdc.Hooks)
}

func (x *scdTx) Store() (scdstore.Store, error) {
	s, err := x.inner.Store()
	if err != nil {
		return nil, err
	}
	st := &scdStore{Store: s, tx: x}
	if h, ok := s.(hookable); ok && !x.t.Invalid() {
		h.SetHooks(&scdc.Hooks{ConflictSearch: st.conflicts, NotificationSearch: st.notificationIDs})
	}
	return st, nil
}

// lockWrites takes the transactor's write lock once per transaction, before
// its first write or write-path mirror search (see SCDTransactor).
func (x *scdTx) lockWrites() {
	if !x.locked {
		x.t.writeMu.Lock()
		x.locked = true
	}
}

func (x *scdTx) unlockWrites() {
	if x.locked {
		x.locked = false
		x.t.writeMu.Unlock()
	}
}

// Commit commits on CRDB, applies the writes to the mirrors and only then
// releases the write lock, whatever the outcome (PerformOperationWithRetries
// starts a new transaction after a failed commit without a rollback).
func (x *scdTx) Commit() error {
	defer x.unlockWrites()
	if err := x.inner.Commit(); err != nil {
		return err
	}
	if err := x.flush(); err != nil {
		// the transaction did commit: report success, stop trusting the mirrors
		atomic.StoreInt32(&x.t.invalid, 1)
	}
	return nil
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
	defer x.unlockWrites()
	x.ops, x.subs = map[scdmodels.ID]*scdmodels.Operation{}, map[scdmodels.ID]*scdmodels.Subscription{}
	return x.inner.Rollback()
}

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

// UpsertOperation is the reference's own (its conflict search and the
// notification ids come from the hooks installed by scdTx.Store); the
// written row is recorded for the mirrors.
func (s *scdStore) UpsertOperation(ctx context.Context, op *scdmodels.Operation, key []scdmodels.OVN) (*scdmodels.Operation, []*scdmodels.Subscription, error) {
	s.tx.lockWrites()
	res, subs, err := s.Store.UpsertOperation(ctx, op, key)
	if err == nil && res != nil {
		s.tx.ops[res.ID] = res
		s.refreshSub(ctx, res.SubscriptionID, res.Owner)
	}
	return res, subs, err
}

// conflicts is UpsertOperation's search (operations.go:337-348: the
// operation's own cells, altitudes and times, ends_at >= now) on the GPU
// mirror, with this transaction's writes overlaid, after searchOperations'
// argument check (operations.go:405-414: the footprint is the operation's
// cells, so only an empty covering can fail).  The transaction takes the
// write lock first and keeps it until its commit has reached the mirrors.
func (s *scdStore) conflicts(ctx context.Context, op *scdmodels.Operation) ([]*scdmodels.Operation, error) {
	if len(op.Cells) == 0 {
		return nil, dsserr.BadRequest("missing cell IDs for query")
	}
	s.tx.lockWrites()
	q := opQuery(op.Cells, op.AltitudeLower, op.AltitudeUpper, op.StartTime, op.EndTime, s.tx.t.Now())
	return s.searchOps(q)
}

// notificationIDs is fetchSubscriptionsForNotification's SELECT DISTINCT
// (subscriptions.go:131-152) on the subscriptions mirror: the subscriptions
// sharing a cell with cells and unexpired (the UPDATE that follows in SQL
// keeps only ends_at >= now), with this transaction's own subscription
// writes overlaid.  The transaction holds the write lock (its operation
// write came first), so no subscription can commit between this read and
// the transaction's own commit unseen.
func (s *scdStore) notificationIDs(ctx context.Context, cells []int64) ([]scdmodels.ID, error) {
	s.tx.lockWrites()
	if len(cells) == 0 {
		return nil, nil // cell_id = ANY('{}'): no rows
	}
	cu := make(s2.CellUnion, len(cells))
	for i, c := range cells {
		cu[i] = s2.CellID(uint64(c))
	}
	t := s.tx.t
	q := Query{Cells: cu, AltLo: negInf, AltHi: posInf, TLo: usOf(t.Now()), THi: timeNullEndQ}
	t.mu.RLock()
	keys, err := t.subs.Search([]Query{q})
	t.mu.RUnlock()
	if err != nil {
		return nil, err
	}
	out := make([]scdmodels.ID, 0, len(keys[0]))
	for _, k := range keys[0] {
		if _, written := s.tx.subs[scdmodels.ID(k)]; !written {
			out = append(out, scdmodels.ID(k))
		}
	}
	for id, sub := range s.tx.subs {
		if sub != nil && subRow(sub).Matches(q) {
			out = append(out, id)
		}
	}
	return out, nil
}

func (s *scdStore) DeleteOperation(ctx context.Context, id scdmodels.ID, owner dssmodels.Owner) (*scdmodels.Operation, []*scdmodels.Subscription, error) {
	s.tx.lockWrites()
	res, subs, err := s.Store.DeleteOperation(ctx, id, owner)
	if err == nil {
		s.tx.ops[id] = nil
		if res != nil {
			s.refreshSub(ctx, res.SubscriptionID, owner)
		}
	}
	return res, subs, err
}

// UpsertSubscription writes under the write lock: its own operation search
// (SQL, subscriptions.go:416) then sees every operation committed before it,
// and every later operation's fan-out sees this subscription.
func (s *scdStore) UpsertSubscription(ctx context.Context, sub *scdmodels.Subscription) (*scdmodels.Subscription, []*scdmodels.Operation, error) {
	s.tx.lockWrites()
	res, ops, err := s.Store.UpsertSubscription(ctx, sub)
	if err == nil && res != nil {
		s.tx.subs[res.ID] = res
	}
	return res, ops, err
}

func (s *scdStore) DeleteSubscription(ctx context.Context, id scdmodels.ID, owner dssmodels.Owner, version scdmodels.Version) (*scdmodels.Subscription, error) {
	s.tx.lockWrites()
	res, err := s.Store.DeleteSubscription(ctx, id, owner, version)
	if err == nil {
		s.tx.subs[id] = nil
	}
	return res, err
}

// opQuery folds searchOperations' bounds (operations.go:394-402) into a
// mirror query: tlo = max(start, now) (COALESCE(ends_at >= start) AND
// ends_at >= now), NULL end -> open.
func opQuery(cells s2.CellUnion, lo, hi *float32, start, end *time.Time, now time.Time) Query {
	tlo := usOf(now)
	if start != nil {
		if st := usOf(*start); st > tlo {
			tlo = st
		}
	}
	return Query{Cells: cells, AltLo: altOr(lo, negInf), AltHi: altOr(hi, posInf), TLo: tlo,
		THi: usOrNull(end, timeNullEndQ)}
}

// searchOps runs q on the operations mirror and maps the keys to rows under
// one read lock (no apply can land between the search and the lookup), with
// the transaction's own writes overlaid.  Results carry no cells, as
// searchOperations' rows do not.
func (s *scdStore) searchOps(q Query) ([]*scdmodels.Operation, error) {
	t := s.tx.t
	t.mu.RLock()
	defer t.mu.RUnlock()
	keys, err := t.ops.Search([]Query{q})
	if err != nil {
		return nil, err
	}
	out := make([]*scdmodels.Operation, 0, len(keys[0]))
	for _, k := range keys[0] {
		id := scdmodels.ID(k)
		if _, written := s.tx.ops[id]; written {
			continue // this transaction's version decides
		}
		if o, ok := t.opRows[id]; ok {
			c := *o
			c.Cells = nil
			out = append(out, &c)
		}
	}
	for _, o := range s.tx.ops {
		if o != nil && opRow(o).Matches(q) {
			c := *o
			c.Cells = nil
			out = append(out, &c)
		}
	}
	return out, nil
}

// SearchOperations replaces searchOperations
// (pkg/scd/store/cockroach/operations.go:374-435): the same argument checks
// and error messages, then
//   cells && cells AND COALESCE(altitude_upper >= lo, true)
//   AND COALESCE(altitude_lower <= hi, true) AND COALESCE(ends_at >= start, true)
//   AND COALESCE(starts_at <= end, true) AND ends_at >= now
// on the GPU mirror.  The owner argument is unused, as in the reference.
func (s *scdStore) SearchOperations(ctx context.Context, v4d *dssmodels.Volume4D, owner dssmodels.Owner) ([]*scdmodels.Operation, error) {
	if s.tx.t.Invalid() {
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
	return s.searchOps(opQuery(cells, v4d.SpatialVolume.AltitudeLo, v4d.SpatialVolume.AltitudeHi, v4d.StartTime,
		v4d.EndTime, s.tx.t.Now()))
}

// SearchSubscriptions replaces the SCD SubscriptionStore.SearchSubscriptions
// (pkg/scd/store/cockroach/subscriptions.go:497-545).  Its LEFT JOIN keeps
// every row of the owner, so the cells only have to be non-empty (quirk Q7):
// the answer is the owner's subscriptions with ends_at >= now.
func (s *scdStore) SearchSubscriptions(ctx context.Context, cells s2.CellUnion, owner dssmodels.Owner) ([]*scdmodels.Subscription, error) {
	if s.tx.t.Invalid() {
		return s.Store.SearchSubscriptions(ctx, cells, owner)
	}
	if len(cells) == 0 {
		return nil, dsserr.BadRequest("no location provided")
	}
	t := s.tx.t
	now := t.Now()
	live := func(sub *scdmodels.Subscription) bool {
		return sub.Owner == owner && sub.EndTime != nil && !sub.EndTime.Before(now)
	}
	t.mu.RLock()
	defer t.mu.RUnlock()
	var out []*scdmodels.Subscription
	for id, sub := range t.subRows {
		if _, written := s.tx.subs[id]; !written && live(sub) {
			c := *sub
			out = append(out, &c)
		}
	}
	for _, sub := range s.tx.subs { // read-your-writes
		if sub != nil && live(sub) {
			c := *sub
			out = append(out, &c)
		}
	}
	// the reference commits this read-only transaction (subscriptions.go:540);
	// here the caller's transaction is left to the caller
	return out, nil
}
