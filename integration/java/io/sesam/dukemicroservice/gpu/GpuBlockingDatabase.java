package io.sesam.dukemicroservice.gpu;

import java.util.ArrayList;
import java.util.BitSet;
import java.util.Collection;
import java.util.HashMap;
import java.util.List;
import java.util.Map;

import no.priv.garshol.duke.Configuration;
import no.priv.garshol.duke.Database;
import no.priv.garshol.duke.Property;
import no.priv.garshol.duke.Record;
import no.priv.garshol.duke.RecordImpl;
import no.priv.garshol.duke.databases.KeyFunction;

/**
 * The index of one pipeline on the GPU: replaces IncrementalLuceneDatabase (App.java:329-342,
 * 450-463) for pipelines GpuEligibility accepts.  index() buffers, commit() upserts the
 * buffered records column-wise (delete-by-ID then add, IncrementalLuceneDatabase.java:
 * 516-517).  Candidates come from dk_match: the device's key-function blocking, or -- no key
 * functions, the reference's own configuration -- IncrementalLuceneDatabase's own query
 * semantics (findCandidateMatches :459-492) run on the device, so findCandidateMatches is not
 * called by GpuProcessor.  Record IDs are interned natively (dk_interner: the identity numbering
 * of both packing paths, the link sink's IDs).  findRecordById is the device index's ID map.
 * Mirrors sesam-duke-microservice_amd/dukehip/processor.py GpuBlockingDatabase.
 *
 * Host memory: a row's Record is held only while the row can still be handed to a listener or
 * looked up -- superseded versions are released at the upsert that supersedes them (not under
 * setOverwrite(true), where they stay candidates), and natively packed batches keep their
 * columns, not Record objects (built per lookup), freed once every row of the batch is gone.
 */
public class GpuBlockingDatabase implements Database {
    private final long ctx;
    private final long ids;                        // dk_interner of record IDs
    private final List<Property> props;            // scored properties, Processor.compare order
    private final List<KeyFunction> keyFunctions;
    private final boolean linkage;
    private final String idProp;
    private final RowStore rows = new RowStore();
    private long[] rowIdent = new long[1024];      // row -> interned record ID
    private final List<Record> pending = new ArrayList<>();
    private final List<Integer> deferred = new ArrayList<>();   // releaseDeferred
    private boolean indexingIsDisabled;
    private boolean overwrite;
    private int transientRow0 = -1;
    private Configuration config;
    private int[] caps = {16};                     // HashMap capacities -> order classes

    /**
     * @param scoredProps  the scored properties in Processor.compare's iteration order
     *                     (comparisonOrder gives it for a data source's records)
     * @param keyFunctions key-function blocking; empty = the reference's Lucene candidate
     *                     semantics on the device (lookup properties and App.configureDatabase's
     *                     knobs, GpuEligibility.lucene)
     * @param devices      the GPUs of this JVM to replicate the index over (dk_create_multi)
     */
    public GpuBlockingDatabase(Configuration config, List<Property> scoredProps,
                               List<KeyFunction> keyFunctions, boolean linkage, int[] devices) {
        this(config, new OrderClasses(scoredProps), keyFunctions, linkage, devices);
    }

    /** The same with the pipeline's Processor.compare order classes (orderClasses). */
    public GpuBlockingDatabase(Configuration config, OrderClasses oc,
                               List<KeyFunction> keyFunctions, boolean linkage, int[] devices) {
        this.config = config;
        List<Property> scoredProps = oc.props;
        this.props = scoredProps;
        this.caps = oc.caps;
        this.keyFunctions = keyFunctions;
        this.linkage = linkage;
        this.idProp = config.getIdentityProperties().iterator().next().getName();
        int n = scoredProps.size();
        int[] cmp = new int[n], q = new int[n], formula = new int[n], tok = new int[n];
        double[] low = new double[n], high = new double[n], minRatio = new double[n];
        for (int i = 0; i < n; i++) {
            GpuEligibility.Opcode op = GpuEligibility.opcode(scoredProps.get(i).getComparator());
            cmp[i] = op.comparator;
            q[i] = op.q;
            formula[i] = op.formula;
            tok[i] = op.tokenizer;
            minRatio[i] = op.minRatio;
            low[i] = scoredProps.get(i).getLowProbability();
            high[i] = scoredProps.get(i).getHighProbability();
        }
        int[] lookup = null;
        int maxHits = 10;
        float minRelevance = 0.9f;
        GpuEligibility.LuceneOptions opts = null;
        if (keyFunctions.isEmpty()) {   // IncrementalLuceneDatabase.findCandidateMatches on the device
            opts = GpuEligibility.lucene(config);
            maxHits = opts.maxSearchHits;
            minRelevance = opts.minRelevance;
            List<Property> lp = config.getLookupProperties();
            lookup = new int[lp.size()];
            for (int i = 0; i < lp.size(); i++) {
                lookup[i] = -1;
                for (int p = 0; p < n; p++)
                    if (scoredProps.get(p).getName().equals(lp.get(i).getName())) lookup[i] = p;
                if (lookup[i] < 0) throw new IllegalArgumentException("lookup property not scored: " + lp.get(i).getName());
            }
        }
        this.ids = DukeHip.internerCreate();
        this.ctx = DukeHip.create(cmp, q, formula, tok, low, high, minRatio, config.getThreshold(),
                                  config.getMaybeThreshold(), linkage ? DukeHip.MODE_LINKAGE : DukeHip.MODE_DEDUP,
                                  keyFunctions.size(), lookup, maxHits, minRelevance,
                                  devices == null || devices.length == 0 ? new int[] {0} : devices,
                                  oc.flatOrders());
        if (opts != null && opts.unmergedStats) DukeHip.luceneSetStats(ctx, DukeHip.LUCENE_STATS_UNMERGED);
    }

    /** IndexWriter.forceMerge of the Lucene source's statistics (dk_lucene_merge): superseded
     *  versions stop counting in maxDoc / docFreq under DUKEHIP_LUCENE_STATS=unmerged. */
    public void forceMerge() {
        if (keyFunctions.isEmpty()) DukeHip.luceneMerge(ctx);
    }

    /**
     * Processor.compare iterates r1.getProperties(): RecordImpl's HashMap key order.  The keys a
     * data source's RecordBuilder inserts -- its columns' properties in column order, then
     * dukeGroupNo (linkage), ID, dukeOriginalEntityId, dukeDatasetId, dukeDeleted
     * (IncrementalDataSource.java:67-98) -- put into a HashMap of the record's capacity give that
     * order; a record missing some values iterates the rest in the same relative order.  The
     * capacity follows the number of keys the record holds (16 up to 12, 32 up to 24, 64 up to
     * 48), so a pipeline whose records can hold more than 12 has several order classes, and
     * each record's class is its capacity's (dk_schema.orders, dk_batch.order_class).
     */
    public static final class OrderClasses {
        final List<Property> props;   // class 0's order: the schema's property order
        final int[] caps;             // ascending capacities, one per class
        final int[][] orders;         // orders[c][k] = index into props of class c's k-th

        OrderClasses(List<Property> props) {
            this.props = props;
            this.caps = new int[] {16};
            int[] id = new int[props.size()];
            for (int i = 0; i < id.length; i++) id[i] = i;
            this.orders = new int[][] {id};
        }

        OrderClasses(List<Property> props, int[] caps, int[][] orders) {
            this.props = props;
            this.caps = caps;
            this.orders = orders;
        }

        /** dk_schema.orders (class-major), or null for one class. */
        int[] flatOrders() {
            if (orders.length <= 1) return null;
            int n = props.size();
            int[] f = new int[orders.length * n];
            for (int c = 0; c < orders.length; c++) System.arraycopy(orders[c], 0, f, c * n, n);
            return f;
        }

        /** the order class of a record holding `keys` properties */
        int classOf(int keys) {
            int cap = 16;
            while (keys > cap * 3 / 4) cap *= 2;
            for (int c = 0; c < caps.length; c++) if (caps[c] == cap) return c;
            throw new DukeHipException(DukeHip.E_UNSUPPORTED, "record of " + keys + " properties");
        }
    }

    /**
     * The order classes of a data source's records: `recordKeys` = every key its records can
     * hold in insertion order (columns' properties, then the synthetic ones incl. dukeDeleted),
     * `minKeys` / `maxKeys` = the fewest / most a record holds (the synthetic ones / all).
     */
    public static OrderClasses orderClasses(Configuration config, List<String> recordKeys, int minKeys, int maxKeys) {
        if (maxKeys > 48)
            throw new IllegalArgumentException("more than 48 record properties: HashMap capacity past 64");
        List<Integer> capList = new ArrayList<>();
        for (int k = minKeys; k <= maxKeys; k++) {
            int cap = 16;
            while (k > cap * 3 / 4) cap *= 2;
            if (!capList.contains(cap)) capList.add(cap);
        }
        if (capList.size() > DukeHip.MAX_ORDER_CLASSES)
            throw new IllegalArgumentException("too many HashMap order classes");
        List<List<Property>> byClass = new ArrayList<>();
        for (int cap : capList) {
            // a bucket of 8 or more keys: a real record map would treeify it, or resize below
            // capacity 64 (HashMap.treeifyBin) -- an order this model does not give (the
            // Python wiring, config.java_hashmap_order, refuses the same pipelines)
            int[] occ = new int[cap];
            for (String k : recordKeys) {
                int h = k.hashCode();
                if (++occ[(h ^ (h >>> 16)) & (cap - 1)] >= 8)
                    throw new IllegalArgumentException("8 record keys in one HashMap bucket at capacity "
                                                       + cap + ": order not modelled");
            }
            // a table of exactly `cap` buckets that never resizes (load factor 100), holding
            // every key a record can have: a record's own keys iterate in this relative order
            Map<String, Boolean> m = new HashMap<>(cap, 100f);
            for (String k : recordKeys) m.put(k, Boolean.TRUE);
            List<Property> out = new ArrayList<>();
            for (String k : m.keySet()) {
                Property p = config.getPropertyByName(k);
                if (p != null && !p.isIdProperty() && !p.isIgnoreProperty()) out.add(p);
            }
            byClass.add(out);
        }
        List<Property> props = byClass.get(0);
        int[] caps = new int[capList.size()];
        int[][] orders = new int[capList.size()][];
        for (int c = 0; c < caps.length; c++) {
            caps[c] = capList.get(c);
            orders[c] = new int[props.size()];
            for (int k = 0; k < props.size(); k++) orders[c][k] = props.indexOf(byClass.get(c).get(k));
        }
        return new OrderClasses(props, caps, orders);
    }

    /**
     * Pipelines whose records hold at most 12 properties: the one order (a HashMap of
     * capacity 16).  A pipeline whose records can hold more has a second order class at least
     * (a record holding 12 or fewer keys still iterates at capacity 16): refused here -- use
     * orderClasses and the OrderClasses constructor, which give every record its class.
     */
    public static List<Property> comparisonOrder(Configuration config, List<String> recordKeys) {
        if (recordKeys.size() > 12)
            throw new IllegalArgumentException(recordKeys.size() + " record keys: several HashMap order "
                                               + "classes, use orderClasses(config, keys, minKeys, maxKeys)");
        return orderClasses(config, recordKeys, recordKeys.size(), recordKeys.size()).props;
    }

    long ctx() { return ctx; }

    long ids() { return ids; }

    Record recordAtRow(int row) { return rows.get(row); }

    long identAtRow(int row) { return rowIdent[row]; }

    List<Property> properties() { return props; }

    boolean indexingIsDisabled() { return indexingIsDisabled; }

    // ---- Database (IncrementalLuceneDatabase.java) ----
    @Override public void setConfiguration(Configuration config) { this.config = config; }

    @Override public void setOverwrite(boolean overwrite) {                  // :99, :515
        this.overwrite = overwrite;
        DukeHip.setOverwrite(ctx, overwrite);
    }

    @Override public boolean isInMemory() { return true; }

    public void setIndexingIsDisabled(boolean disabled) {           // :95
        indexingIsDisabled = disabled;
        if (!disabled) dropTransient();
    }

    @Override public void index(Record record) {                     // :498-503
        if (!indexingIsDisabled) pending.add(record);
    }

    @Override public void commit() {                                 // :146-165
        List<Record> batch = new ArrayList<>(pending);
        pending.clear();
        indexBatch(batch, false);
    }

    @Override public Record findRecordById(String id) {              // :170-180
        long ident = DukeHip.internerFind(ids, id);
        if (ident < 0) return null;
        int row = DukeHip.rowOfIdent(ctx, ident);
        return row < 0 ? null : rows.get(row);
    }

    @Override public Collection<Record> findCandidateMatches(Record record) {
        throw new UnsupportedOperationException("candidates come from dk_match (GpuProcessor)");
    }

    @Override public void close() {
        DukeHip.destroy(ctx);
        rows.clear();
        DukeHip.internerDestroy(ids);
    }

    /** Records handed to index() before a deduplicate batch, committed with it. */
    List<Record> takePending() {
        List<Record> p = new ArrayList<>(pending);
        pending.clear();
        return p;
    }

    void dropTransient() {
        if (transientRow0 >= 0) {
            DukeHip.dropTransient(ctx);
            rows.truncate(transientRow0);
            transientRow0 = -1;
        }
    }

    /** Every record the index holds, live versions (GpuProcessor's hand-over to stock Duke). */
    List<Record> liveRecords() {
        List<Record> out = new ArrayList<>();
        for (int r = 0; r < rows.size(); r++) {
            if (transientRow0 >= 0 && r >= transientRow0) break;
            Record rec = rows.get(r);
            if (rec != null && (overwrite || DukeHip.rowOfIdent(ctx, rowIdent[r]) == r)) out.add(rec);
        }
        return out;
    }

    private long[] intern(List<Record> batch) {
        int n = batch.size();
        String[] id = new String[n];
        for (int i = 0; i < n; i++) {
            id[i] = batch.get(i).getValue(idProp);
            if (id[i] == null) throw new RuntimeException("record without ID property");
        }
        int[] off = new int[n + 1];
        char[] units = arena(id, off, null);
        return DukeHip.internerIntern(ids, off, units);
    }

    /** Rows the batch's IDs map to before the upsert: they are superseded by it. */
    private int[] previousRows(long[] ident) {
        int[] prev = new int[ident.length];
        for (int i = 0; i < ident.length; i++) prev[i] = overwrite ? -1 : DukeHip.rowOfIdent(ctx, ident[i]);
        return prev;
    }

    private void afterUpsert(long[] ident, int[] prev, int[] assigned, boolean asTransient) {
        int row0 = assigned.length > 0 ? assigned[0] : rows.size();
        if (rowIdent.length < row0 + ident.length)
            rowIdent = java.util.Arrays.copyOf(rowIdent, Math.max(2 * rowIdent.length, row0 + ident.length));
        System.arraycopy(ident, 0, rowIdent, row0, ident.length);
        if (asTransient) return;
        for (int i = 0; i < prev.length; i++) if (prev[i] >= 0) rows.release(prev[i]);
        // an ID twice in this batch: the earlier copy is superseded by the later one, but it is
        // still a query record of this batch -- released after the replay (releaseDeferred)
        Map<Long, Integer> last = new HashMap<>();
        for (int i = 0; i < ident.length; i++) {
            Integer before = last.put(ident[i], assigned[i]);
            if (before != null && !overwrite) deferred.add(before);
        }
    }

    /** After a batch's replay: the rows its later copies superseded drop their Records. */
    void releaseDeferred() {
        for (int r : deferred) rows.release(r);
        deferred.clear();
    }

    /** Packs `batch` column-wise and upserts it (dk_upsert, or dk_upsert_transient). */
    int[] indexBatch(List<Record> batch, boolean asTransient) {
        int n = batch.size();
        if (n == 0) return new int[0];
        long[] ident = intern(batch);
        byte[] group = linkage ? new byte[n] : null;
        byte[] deleted = new byte[n];
        for (int i = 0; i < n; i++) {
            Record r = batch.get(i);
            deleted[i] = (byte) ("true".equals(r.getValue("dukeDeleted")) ? 1 : 0);
            if (linkage) {
                String g = r.getValue("dukeGroupNo");
                if (!"1".equals(g) && !"2".equals(g))   // IncrementalLuceneDatabase.java:469-471
                    throw new RuntimeException("The 'dukeGroupNo' property was missing or empty!");
                group[i] = (byte) Integer.parseInt(g);
            }
        }
        int np = props.size(), nk = keyFunctions.size();
        int[][] offsets = new int[np][], keyOffsets = new int[nk][];
        char[][] units = new char[np][], keyUnits = new char[nk][];
        byte[][] present = new byte[np][];
        for (int p = 0; p < np; p++) {
            String[] vals = new String[n];
            for (int i = 0; i < n; i++) {
                Collection<String> vs = batch.get(i).getValues(props.get(p).getName());
                if (vs != null && vs.size() > 1)
                    throw new DukeHipException(DukeHip.E_UNSUPPORTED, "more than one value for " + props.get(p).getName());
                vals[i] = vs == null || vs.isEmpty() ? null : vs.iterator().next();
            }
            present[p] = new byte[n];
            offsets[p] = new int[n + 1];
            units[p] = arena(vals, offsets[p], present[p]);
        }
        for (int k = 0; k < nk; k++) {
            String[] keys = new String[n];
            for (int i = 0; i < n; i++) keys[i] = keyFunctions.get(k).makeKey(batch.get(i));
            keyOffsets[k] = new int[n + 1];
            keyUnits[k] = arena(keys, keyOffsets[k], null);
        }
        byte[] orderClass = null;
        if (caps.length > 1) {   // Processor.compare follows each query record's HashMap order
            OrderClasses oc = new OrderClasses(props, caps, null);
            orderClass = new byte[n];
            for (int i = 0; i < n; i++) orderClass[i] = (byte) oc.classOf(batch.get(i).getProperties().size());
        }
        int[] prev = asTransient ? new int[0] : previousRows(ident);
        int[] assigned = DukeHip.upsert(ctx, asTransient, n, ident, group, deleted, offsets, units,
                                        present, keyOffsets, keyUnits, orderClass);
        if (asTransient && transientRow0 < 0) transientRow0 = rows.size();
        rows.appendRecords(batch);
        afterUpsert(ident, prev, assigned, asTransient);
        return assigned;
    }

    /**
     * The POSTed body of data source `src`, packed natively (dk_pack_json: no Gson tree, no
     * Record objects) and upserted.  Returns the batch's rows; DukeHipException E_UNSUPPORTED
     * when the native reader declines the body (the caller then takes the Record path).
     */
    int[] indexJson(byte[] body, JsonSource src, boolean asTransient) {
        if (caps.length > 1)   // the native packer does not count a record's properties
            throw new DukeHipException(DukeHip.E_UNSUPPORTED, "several HashMap order classes");
        long packed = DukeHip.packJson(ids, body, src.datasetId, src.groupNo, src.columnNames,
                                       src.columnProp, src.columnCleaner, props.size(), src.keyParts);
        int n = DukeHip.packedSize(packed);
        if (n == 0) {
            DukeHip.freePacked(packed);
            return new int[0];
        }
        if (linkage && src.groupNo == 0) {
            DukeHip.freePacked(packed);
            throw new RuntimeException("The 'dukeGroupNo' property was missing or empty!");
        }
        long[] ident = DukeHip.packedIdent(packed);
        int[] prev = asTransient ? new int[0] : previousRows(ident);
        int[] assigned;
        try {
            assigned = DukeHip.upsertPacked(ctx, packed, asTransient);
        } catch (RuntimeException e) {
            DukeHip.freePacked(packed);
            throw e;
        }
        if (asTransient && transientRow0 < 0) transientRow0 = rows.size();
        rows.appendPacked(new PackedBatch(packed, n, src, props));
        afterUpsert(ident, prev, assigned, asTransient);
        return assigned;
    }

    /** Processor.compare of two records by value (dk_compare_values; the index is untouched). */
    double compareValues(Record r1, Record r2) {
        String[] a = new String[props.size()], b = new String[props.size()];
        for (int p = 0; p < props.size(); p++) {
            a[p] = single(r1, props.get(p).getName());
            b[p] = single(r2, props.get(p).getName());
        }
        return DukeHip.compareValues(ctx, a, b);
    }

    private static String single(Record r, String prop) {
        Collection<String> vs = r.getValues(prop);
        if (vs != null && vs.size() > 1) throw new IllegalStateException("more than one value: not GPU-eligible");
        return vs == null || vs.isEmpty() ? null : vs.iterator().next();
    }

    static char[] arena(String[] vals, int[] off, byte[] present) {
        int total = 0;
        for (String v : vals) total += v == null ? 0 : v.length();
        char[] out = new char[total];
        int at = 0;
        for (int i = 0; i < vals.length; i++) {
            off[i] = at;
            if (vals[i] != null) {
                vals[i].getChars(0, vals[i].length(), out, at);
                at += vals[i].length();
            }
            if (present != null) present[i] = (byte) (vals[i] != null ? 1 : 0);
        }
        off[vals.length] = at;
        return out;
    }

    /**
     * A data source as dk_pack_json reads it (the microservice's IncrementalDataSource):
     * dataset id, RecordLinkage group (0 = deduplication), its columns (JSON attribute, scored
     * property index or -1, DukeHip.CLEAN_* cleaner) in data-source order, and the key
     * functions as parts (PartsKeyFunction.parts(); null with the Lucene source).
     */
    public static final class JsonSource {
        final String datasetId;
        final int groupNo;
        final String[] columnNames;
        final int[] columnProp, columnCleaner;
        final int[][] keyParts;

        public JsonSource(String datasetId, int groupNo, String[] columnNames, int[] columnProp,
                          int[] columnCleaner, int[][] keyParts) {
            this.datasetId = datasetId;
            this.groupNo = groupNo;
            this.columnNames = columnNames;
            this.columnProp = columnProp;
            this.columnCleaner = columnCleaner;
            this.keyParts = keyParts;
        }
    }

    /** A natively packed batch: its columns stay in native memory, Records are built per row
     *  on lookup (IncrementalDataSource.java:67-98's record shape). */
    static final class PackedBatch {
        final long handle;
        final int n;
        final JsonSource src;
        final List<Property> props;
        String[][] values;     // per scored property, fetched on the first lookup
        String[] id, entityId;
        byte[] deleted;

        PackedBatch(long handle, int n, JsonSource src, List<Property> props) {
            this.handle = handle;
            this.n = n;
            this.src = src;
            this.props = props;
        }

        Record record(int i) {
            if (values == null) {
                values = new String[props.size()][];
                for (int p = 0; p < props.size(); p++) values[p] = DukeHip.packedValues(handle, p);
                id = DukeHip.packedIds(handle);
                entityId = DukeHip.packedEntityIds(handle);
                deleted = DukeHip.packedDeleted(handle);
            }
            RecordImpl r = new RecordImpl();   // [Duke 1.2, recalled] ModifiableRecord
            for (int p = 0; p < props.size(); p++)
                if (values[p][i] != null) r.addValue(props.get(p).getName(), values[p][i]);
            if (src.groupNo != 0) r.addValue("dukeGroupNo", Integer.toString(src.groupNo));
            r.addValue("ID", id[i]);
            r.addValue("dukeOriginalEntityId", entityId[i]);
            r.addValue("dukeDatasetId", src.datasetId);
            if (deleted[i] != 0) r.addValue("dukeDeleted", "true");
            return r;
        }

        void free() { DukeHip.freePacked(handle); }
    }

    /** row -> Record over segments of Record batches and packed batches; released rows drop
     *  their Record, and a segment whose rows are all released drops its payload. */
    static final class RowStore {
        private static final class Segment {
            final int row0, n;
            List<Record> records;     // Record path
            PackedBatch packed;       // native path
            final BitSet released = new BitSet();
            int live;

            Segment(int row0, int n) {
                this.row0 = row0;
                this.n = n;
                this.live = n;
            }
        }

        private final List<Segment> segs = new ArrayList<>();
        private int size;

        int size() { return size; }

        void appendRecords(List<Record> batch) {
            Segment s = new Segment(size, batch.size());
            s.records = new ArrayList<>(batch);
            segs.add(s);
            size += batch.size();
        }

        void appendPacked(PackedBatch b) {
            Segment s = new Segment(size, b.n);
            s.packed = b;
            segs.add(s);
            size += b.n;
        }

        private Segment seg(int row) {
            int lo = 0, hi = segs.size();
            while (hi - lo > 1) {
                int mid = (lo + hi) >>> 1;
                if (segs.get(mid).row0 <= row) lo = mid;
                else hi = mid;
            }
            return segs.get(lo);
        }

        Record get(int row) {
            if (row < 0 || row >= size) return null;
            Segment s = seg(row);
            int i = row - s.row0;
            if (s.released.get(i)) return null;
            return s.records != null ? s.records.get(i) : s.packed.record(i);
        }

        void release(int row) {
            if (row < 0 || row >= size) return;
            Segment s = seg(row);
            int i = row - s.row0;
            if (s.released.get(i)) return;
            s.released.set(i);
            if (s.records != null) s.records.set(i, null);
            if (--s.live == 0) drop(s);
        }

        private static void drop(Segment s) {
            s.records = null;
            if (s.packed != null) {
                s.packed.free();
                s.packed = null;
            }
        }

        void truncate(int n) {
            while (!segs.isEmpty() && segs.get(segs.size() - 1).row0 >= n) drop(segs.remove(segs.size() - 1));
            size = n;
        }

        void clear() {
            for (Segment s : segs) drop(s);
            segs.clear();
            size = 0;
        }
    }
}
