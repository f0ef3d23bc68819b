package gpu

/*
#include <stdlib.h>
#include "dssgpu.h"
*/
import "C"

import (
	"unsafe"

	"github.com/golang/geo/s2"
	"github.com/interuss/dss/pkg/geo"
	dssmodels "github.com/interuss/dss/pkg/models"
)

// Which package's sentinel a failed covering returns: the reference defines
// the same messages twice, as distinct error values, in pkg/geo (s2.go:37-39,
// Covering / AreaToCellIDs) and in pkg/models (geo.go:36-38, the
// GeoPolygon / GeoCircle methods).  Callers compare with ==, so the binding
// returns the value of the package the replaced function lives in: pkg/geo's
// for point lists and area strings, pkg/models' for polygons and circles.
type errorSet int

const (
	geoErrors errorSet = iota
	modelErrors
)

func errorsFor(kind int32) errorSet {
	if kind == KindPoints {
		return geoErrors
	}
	return modelErrors
}

// statusErr maps a DSSG_ST_* status to the reference's error value
// (INTEGRATION.md, "Error mapping").
func statusErr(set errorSet, st C.int32_t, areaKm2 C.double) error {
	switch st {
	case C.DSSG_ST_OK:
		return nil
	case C.DSSG_ST_AREA_TOO_LARGE:
		return geo.NewErrAreaTooLarge(float64(areaKm2)) // pkg/geo/s2.go:112-116, exact message
	case C.DSSG_ST_ODD_COORDS:
		return geo.ErrOddNumberOfCoordinatesInAreaString
	case C.DSSG_ST_NOT_ENOUGH_POINTS:
		if set == modelErrors {
			return dssmodels.ErrNotEnoughPointsInPolygon
		}
		return geo.ErrNotEnoughPointsInPolygon
	case C.DSSG_ST_RADIUS:
		return dssmodels.ErrRadiusMustBeLargerThan0
	default: // DSSG_ST_BAD_COORD_SET
		if set == modelErrors {
			return dssmodels.ErrBadCoordSet
		}
		return geo.ErrBadCoordSet
	}
}

// Footprint is one covering request: a polygon / point list (lat, lng in
// degrees) or a circle (one centre, radius in metres).
type Footprint struct {
	Kind    int32 // DSSG_KIND_POLYGON, DSSG_KIND_CIRCLE, DSSG_KIND_POINTS
	Lat     []float64
	Lng     []float64
	RadiusM float32
}

// Kinds (dssgpu.h).
const (
	KindPolygon = int32(C.DSSG_KIND_POLYGON)
	KindCircle  = int32(C.DSSG_KIND_CIRCLE)
	KindPoints  = int32(C.DSSG_KIND_POINTS)
)

// CoverBatch covers a batch of footprints in one call (dssg_cover_batch):
// the per-footprint results are the cells and error the replaced Go function
// would return for each, in order.
func CoverBatch(fps []Footprint) ([]s2.CellUnion, []error, error) {
	n := len(fps)
	if n == 0 {
		return nil, nil, nil
	}
	c, err := getCtx()
	if err != nil {
		return nil, nil, err
	}
	defer putCtx(c)
	kind := make([]C.int32_t, n)
	voff := make([]C.int64_t, n+1)
	radius := make([]C.float, n)
	for i, f := range fps {
		kind[i] = C.int32_t(f.Kind)
		voff[i+1] = voff[i] + C.int64_t(len(f.Lat))
		radius[i] = C.float(f.RadiusM)
	}
	nv := int(voff[n])
	lat := make([]C.double, nv+1)
	lng := make([]C.double, nv+1)
	for i, f := range fps {
		for k := range f.Lat {
			lat[int(voff[i])+k] = C.double(f.Lat[k])
			lng[int(voff[i])+k] = C.double(f.Lng[k])
		}
	}
	offs := make([]C.int64_t, n+1)
	status := make([]C.int32_t, n)
	area := make([]C.double, n)
	cells := make([]uint64, 64*n)
	for {
		var needed C.int64_t
		rc := C.dssg_cover_batch(c.c, C.int64_t(n), &kind[0], &voff[0], &lat[0], &lng[0], &radius[0], &offs[0],
			(*C.uint64_t)(unsafe.Pointer(&cells[0])), C.int64_t(len(cells)), &needed, &status[0], &area[0])
		if rc == C.DSSG_ERR_CAPACITY {
			cells = make([]uint64, int(needed)+1)
			continue
		}
		if rc != C.DSSG_OK {
			return nil, nil, c.err("dssg_cover_batch", rc)
		}
		break
	}
	out := make([]s2.CellUnion, n)
	errs := make([]error, n)
	for i := range fps {
		if e := statusErr(errorsFor(fps[i].Kind), status[i], area[i]); e != nil {
			errs[i] = e
			continue
		}
		out[i] = toCellUnion(cells[offs[i]:offs[i+1]])
	}
	return out, errs, nil
}

func coverOne(f Footprint) (s2.CellUnion, error) {
	cu, errs, err := CoverBatch([]Footprint{f})
	if err != nil {
		return nil, err
	}
	if errs[0] != nil {
		return nil, errs[0]
	}
	return cu[0], nil
}

// CoveringDegrees replaces geo.Covering (pkg/geo/s2.go:99-122) for the
// points s2.PointFromLatLng(s2.LatLngFromDegrees(lat[i], lng[i])) -- the form
// every reference caller builds its points in (AreaToCellIDs, GeoPolygon) --
// bit for bit.
func CoveringDegrees(lat, lng []float64) (s2.CellUnion, error) {
	return coverOne(Footprint{Kind: KindPoints, Lat: lat, Lng: lng})
}

// Covering is geo.Covering for callers that only hold s2.Points: the points
// go through their lat/lng in degrees, so a point that is not exactly the
// image of a degree pair may land on a neighbouring bit pattern (use
// CoveringDegrees where the degrees are at hand).
func Covering(points []s2.Point) (s2.CellUnion, error) {
	lat, lng := make([]float64, len(points)), make([]float64, len(points))
	for i, p := range points {
		ll := s2.LatLngFromPoint(p)
		lat[i], lng[i] = ll.Lat.Degrees(), ll.Lng.Degrees()
	}
	return CoveringDegrees(lat, lng)
}

// AreaToCellIDs replaces geo.AreaToCellIDs (pkg/geo/s2.go:129-166): the
// string is parsed by the library with the reference's own rules (comma
// count before parsing, bufio splitAtComma tokens, ParseFloat).
func AreaToCellIDs(area string) (s2.CellUnion, error) {
	c, err := getCtx()
	if err != nil {
		return nil, err
	}
	defer putCtx(c)
	cs := C.CString(area)
	defer C.free(unsafe.Pointer(cs))
	cells := make([]uint64, 256)
	for {
		var needed C.int64_t
		var st C.int32_t
		var km2 C.double
		rc := C.dssg_area_to_cell_ids(c.c, cs, (*C.uint64_t)(unsafe.Pointer(&cells[0])), C.int64_t(len(cells)),
			&needed, &st, &km2)
		if rc == C.DSSG_ERR_CAPACITY {
			cells = make([]uint64, int(needed)+1)
			continue
		}
		if rc != C.DSSG_OK {
			return nil, c.err("dssg_area_to_cell_ids", rc)
		}
		if e := statusErr(geoErrors, st, km2); e != nil {
			return nil, e
		}
		return toCellUnion(cells[:needed]), nil
	}
}

// Polygon is a models.Geometry whose covering runs on the GPU; it replaces
// (*models.GeoPolygon).CalculateCovering (pkg/models/geo.go:252-268).
type Polygon struct{ *dssmodels.GeoPolygon }

// CalculateCovering implements models.Geometry.
func (p Polygon) CalculateCovering() (s2.CellUnion, error) {
	if p.GeoPolygon == nil {
		return nil, dssmodels.ErrBadCoordSet
	}
	f := Footprint{Kind: KindPolygon, Lat: make([]float64, len(p.Vertices)), Lng: make([]float64, len(p.Vertices))}
	for i, v := range p.Vertices {
		f.Lat[i], f.Lng[i] = v.Lat, v.Lng
	}
	return coverOne(f)
}

// Circle is a models.Geometry whose covering runs on the GPU; it replaces
// (*models.GeoCircle).CalculateCovering (pkg/models/geo.go:224-239).
type Circle struct{ *dssmodels.GeoCircle }

// CalculateCovering implements models.Geometry.
func (g Circle) CalculateCovering() (s2.CellUnion, error) {
	f := Footprint{Kind: KindCircle, Lat: []float64{g.Center.Lat}, Lng: []float64{g.Center.Lng}, RadiusM: g.RadiusMeter}
	return coverOne(f)
}

// Geometry wraps a footprint decoded by the reference's proto converters
// (models.Volume4DFromSCDProto etc.) so its covering runs on the GPU; other
// Geometry implementations (precomputed cells, GeometryFunc) pass through.
func Geometry(g dssmodels.Geometry) dssmodels.Geometry {
	switch x := g.(type) {
	case *dssmodels.GeoPolygon:
		return Polygon{x}
	case *dssmodels.GeoCircle:
		return Circle{x}
	default:
		return g
	}
}

// OnGPU rewrites a volume's footprint in place (see Geometry).
func OnGPU(v4 *dssmodels.Volume4D) *dssmodels.Volume4D {
	if v4 != nil && v4.SpatialVolume != nil && v4.SpatialVolume.Footprint != nil {
		v4.SpatialVolume.Footprint = Geometry(v4.SpatialVolume.Footprint)
	}
	return v4
}
