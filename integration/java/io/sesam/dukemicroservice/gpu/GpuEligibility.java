package io.sesam.dukemicroservice.gpu;

import java.lang.reflect.Field;

import no.priv.garshol.duke.Comparator;
import no.priv.garshol.duke.Configuration;
import no.priv.garshol.duke.Property;

/**
 * Whether a pipeline can run on the GPU, and the DK_CMP_* opcode of each comparator
 * (include/dukehip.h; the same table as dukehip/config.py COMPARATOR_CLASSES).  A pipeline is
 * GPU-eligible as a whole: any comparator without a kernel keeps it on stock Duke, so there is
 * no silent divergence.  The bean parameters ConfigLoader set (QGramComparator q / formula /
 * tokenizer, NumericComparator min-ratio) are read back by field name [Duke 1.2, recalled].
 */
public final class GpuEligibility {
    private GpuEligibility() {}

    public static final class Opcode {
        public final int comparator, q, formula, tokenizer;
        public final double minRatio;

        Opcode(int comparator, int q, int formula, int tokenizer, double minRatio) {
            this.comparator = comparator;
            this.q = q;
            this.formula = formula;
            this.tokenizer = tokenizer;
            this.minRatio = minRatio;
        }
    }

    /**
     * Whether the pipeline can run on the GPU.  keyFunctions empty = the reference's own
     * database (IncrementalLuceneDatabase), whose candidate semantics the device then runs
     * (dk_schema.lucene): eligible with the database knobs App.configureDatabase reads
     * (App.java:550-563) unless FUZZY_SEARCH=true meets a tokenized lookup comparator
     * (FuzzyQuery, IncrementalLuceneDatabase.java:311-315), a lookup property is
     * Lookup.REQUIRED (MUST clauses, :487-488) or MAX_SEARCH_HITS exceeds 100.
     */
    public static boolean check(Configuration config, boolean keyFunctions) {
        try {
            for (Property p : config.getProperties())
                if (!p.isIdProperty() && !p.isIgnoreProperty()) opcode(p.getComparator());
            if (!keyFunctions) lucene(config);
            return true;
        } catch (IllegalArgumentException e) {
            return false;
        }
    }

    /** The Lucene candidate source's settings (App.configureDatabase, App.java:550-563). */
    public static final class LuceneOptions {
        public final int maxSearchHits;
        public final float minRelevance;
        /** DUKEHIP_LUCENE_STATS=unmerged: superseded versions keep counting in maxDoc / docFreq
         *  (Lucene 4's deleted-but-unmerged documents) -- dk_lucene_set_stats */
        public final boolean unmergedStats;

        LuceneOptions(int maxSearchHits, float minRelevance, boolean unmergedStats) {
            this.maxSearchHits = maxSearchHits;
            this.minRelevance = minRelevance;
            this.unmergedStats = unmergedStats;
        }
    }

    public static LuceneOptions lucene(Configuration config) {
        float minRelevance = 0.9f;
        boolean fuzzy = false;
        int maxHits = 10;
        if (System.getenv("MIN_RELEVANCE") != null) minRelevance = Float.parseFloat(System.getenv("MIN_RELEVANCE"));
        if (System.getenv("FUZZY_SEARCH") != null) fuzzy = Boolean.parseBoolean(System.getenv("FUZZY_SEARCH"));
        if (System.getenv("MAX_SEARCH_HITS") != null) maxHits = Integer.parseInt(System.getenv("MAX_SEARCH_HITS"));
        if (maxHits < 1 || maxHits > 100) throw new IllegalArgumentException("MAX_SEARCH_HITS " + maxHits);
        if (config.getLookupProperties().isEmpty()) throw new IllegalArgumentException("no lookup properties");
        // a GeopositionComparator as the only lookup property: the reference's geo search
        // raises (IncrementalLuceneDatabase.java:433-441, 460-463) -- stock Duke keeps it
        if (config.getLookupProperties().size() == 1) {
            Comparator only = config.getLookupProperties().iterator().next().getComparator();
            if (only != null && only.getClass().getName().equals("no.priv.garshol.duke.comparators.GeopositionComparator"))
                throw new IllegalArgumentException("GeopositionComparator as the only lookup property");
        }
        for (Property p : config.getLookupProperties()) {
            if (p.getLookupBehaviour() == Property.Lookup.REQUIRED)
                throw new IllegalArgumentException("Lookup.REQUIRED: MUST clauses are not GPU-eligible");
            Comparator c = p.getComparator();
            if (fuzzy && c != null && c.isTokenized())
                throw new IllegalArgumentException("FUZZY_SEARCH over a tokenized comparator");
        }
        String stats = System.getenv("DUKEHIP_LUCENE_STATS");
        if (stats != null && !stats.equals("merged") && !stats.equals("unmerged"))
            throw new IllegalArgumentException("DUKEHIP_LUCENE_STATS " + stats);
        return new LuceneOptions(maxHits, minRelevance, "unmerged".equals(stats));
    }

    public static Opcode opcode(Comparator c) {
        if (c == null) return new Opcode(DukeHip.CMP_NONE, 2, 0, 0, 0.0);
        String name = c.getClass().getName();
        switch (name) {
            case "no.priv.garshol.duke.comparators.Levenshtein":
                return new Opcode(DukeHip.CMP_LEVENSHTEIN, 2, 0, 0, 0.0);
            case "no.priv.garshol.duke.comparators.JaroWinkler":
                return new Opcode(DukeHip.CMP_JAROWINKLER, 2, 0, 0, 0.0);
            case "no.priv.garshol.duke.comparators.ExactComparator":
                return new Opcode(DukeHip.CMP_EXACT, 2, 0, 0, 0.0);
            case "no.priv.garshol.duke.comparators.WeightedLevenshtein":
                return new Opcode(DukeHip.CMP_WEIGHTED_LEVENSHTEIN, 2, 0, 0, 0.0);
            case "no.priv.garshol.duke.comparators.GeopositionComparator":
                // max-distance (meters) travels in the double parameter (dk_property.min_ratio)
                return new Opcode(DukeHip.CMP_GEOPOSITION, 2, 0, 0, ((Number) field(c, "maxdist")).doubleValue());
            case "no.priv.garshol.duke.comparators.NumericComparator":
                return new Opcode(DukeHip.CMP_NUMERIC, 2, 0, 0, ((Number) field(c, "minratio")).doubleValue());
            case "no.priv.garshol.duke.comparators.QGramComparator": {
                int q = ((Number) field(c, "q")).intValue();
                int formula = ordinal(field(c, "formula"), "OVERLAP", "JACCARD", "DICE");
                int tok = ordinal(field(c, "tokenizer"), "BASIC", "POSITIONAL", "ENDS");
                if (q < 1 || q > 4 || (tok == 1 && q > 3)) throw new IllegalArgumentException("q");
                return new Opcode(DukeHip.CMP_QGRAM, q, formula, tok, 0.0);
            }
            case "no.priv.garshol.duke.comparators.DiceCoefficientComparator":
            case "no.priv.garshol.duke.comparators.JaccardIndexComparator": {
                Object sub = field(c, "subcomp");
                if (sub != null && !sub.getClass().getName().equals("no.priv.garshol.duke.comparators.ExactComparator"))
                    throw new IllegalArgumentException("sub-comparator");
                return new Opcode(name.endsWith("DiceCoefficientComparator") ? DukeHip.CMP_DICE_TOKENS
                                                                           : DukeHip.CMP_JACCARD_TOKENS, 2, 0, 0, 0.0);
            }
            default:
                throw new IllegalArgumentException("no GPU kernel for " + name);
        }
    }

    private static Object field(Object o, String name) {
        for (Class<?> k = o.getClass(); k != null; k = k.getSuperclass()) {
            try {
                Field f = k.getDeclaredField(name);
                f.setAccessible(true);
                return f.get(o);
            } catch (NoSuchFieldException e) {
                // superclass next
            } catch (IllegalAccessException e) {
                throw new IllegalArgumentException(e);
            }
        }
        throw new IllegalArgumentException("field " + name);
    }

    private static int ordinal(Object enumValue, String... names) {
        String s = String.valueOf(enumValue);
        for (int i = 0; i < names.length; i++)
            if (names[i].equals(s)) return i;
        throw new IllegalArgumentException(s);
    }
}
