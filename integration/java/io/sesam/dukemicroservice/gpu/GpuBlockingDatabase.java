package io.sesam.dukemicroservice.gpu;

import java.util.ArrayList;
import java.util.Collection;
import java.util.HashMap;
import java.util.List;
import java.util.Map;

import no.priv.garshol.duke.Configuration;
import no.priv.garshol.duke.Database;
import no.priv.garshol.duke.Property;
import no.priv.garshol.duke.Record;
import no.priv.garshol.duke.databases.KeyFunction;

/**
 * The index of one pipeline on the GPU: replaces IncrementalLuceneDatabase (App.java:329-342,
 * 450-463) for pipelines GpuEligibility accepts.  index() buffers, commit() upserts the
 * buffered records column-wise (delete-by-ID then add, IncrementalLuceneDatabase.java:
 * 516-517), findRecordById is served from the host-side ID -> row map.  Candidate generation
 * is key-function blocking on the device (dk_match), so findCandidateMatches is not called by
 * GpuProcessor.  Mirrors sesam-duke-microservice_amd/dukehip/processor.py GpuBlockingDatabase.
 */
public class GpuBlockingDatabase implements Database {
    private final long ctx;
    private final List<Property> props;           // scored properties, Processor.compare order
    private final List<KeyFunction> keyFunctions;
    private final int mode;
    private final boolean linkage;
    private final List<Record> pending = new ArrayList<>();
    private final List<Record> rows = new ArrayList<>();            // row -> Record
    private final Map<String, Integer> liveRow = new HashMap<>();   // ID -> live row
    private final Map<String, Long> idents = new HashMap<>();       // ID -> dense identity
    private boolean indexingIsDisabled;
    private int transientRow0 = -1;
    private Configuration config;

    public GpuBlockingDatabase(Configuration config, List<Property> scoredProps,
                               List<KeyFunction> keyFunctions, boolean linkage, int device) {
        this.config = config;
        this.props = scoredProps;
        this.keyFunctions = keyFunctions;
        this.linkage = linkage;
        this.mode = linkage ? DukeHip.MODE_LINKAGE : DukeHip.MODE_DEDUP;
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
        this.ctx = DukeHip.create(cmp, q, formula, tok, low, high, minRatio, config.getThreshold(),
                                  config.getMaybeThreshold(), mode, keyFunctions.size(), device);
    }

    long ctx() { return ctx; }

    Record recordAtRow(int row) { return rows.get(row); }

    boolean indexingIsDisabled() { return indexingIsDisabled; }

    // ---- Database (IncrementalLuceneDatabase.java) ----
    @Override public void setConfiguration(Configuration config) { this.config = config; }

    @Override public void setOverwrite(boolean overwrite) { DukeHip.setOverwrite(ctx, overwrite); }

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
        Integer row = liveRow.get(id);
        return row == null ? null : rows.get(row);
    }

    @Override public Collection<Record> findCandidateMatches(Record record) {
        throw new UnsupportedOperationException("candidates come from dk_match (GpuProcessor)");
    }

    @Override public void close() { DukeHip.destroy(ctx); }

    /** Records handed to index() before a deduplicate batch, committed with it. */
    List<Record> takePending() {
        List<Record> p = new ArrayList<>(pending);
        pending.clear();
        return p;
    }

    void dropTransient() {
        if (transientRow0 >= 0) {
            DukeHip.dropTransient(ctx);
            while (rows.size() > transientRow0) rows.remove(rows.size() - 1);
            transientRow0 = -1;
        }
    }

    /** Packs `batch` column-wise and upserts it (dk_upsert, or dk_upsert_transient). */
    int[] indexBatch(List<Record> batch, boolean asTransient) {
        int n = batch.size();
        if (n == 0) return new int[0];
        String idProp = config.getIdentityProperties().iterator().next().getName();
        long[] ident = new long[n];
        byte[] group = linkage ? new byte[n] : null;
        byte[] deleted = new byte[n];
        for (int i = 0; i < n; i++) {
            Record r = batch.get(i);
            String id = r.getValue(idProp);
            Long v = idents.get(id);
            if (v == null) {
                v = (long) idents.size();
                idents.put(id, v);
            }
            ident[i] = v;
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
                    throw new IllegalStateException("more than one value: not GPU-eligible");
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
        int[] assigned = DukeHip.upsert(ctx, asTransient, n, ident, group, deleted, offsets, units,
                                        present, keyOffsets, keyUnits);
        if (asTransient && transientRow0 < 0) transientRow0 = rows.size();
        rows.addAll(batch);
        if (!asTransient)
            for (int i = 0; i < n; i++) liveRow.put(batch.get(i).getValue(idProp), assigned[i]);
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

    private static char[] arena(String[] vals, int[] off, byte[] present) {
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
}
